"""paddle_operator_amd.api"""
