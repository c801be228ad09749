"""paddle_operator_amd.utils"""
