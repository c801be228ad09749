"""paddle_operator_amd.controller"""
