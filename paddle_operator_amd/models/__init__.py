"""paddle_operator_amd.models"""
