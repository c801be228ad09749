"""paddle_operator_amd.launch"""
