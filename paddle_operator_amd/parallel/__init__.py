"""paddle_operator_amd.parallel"""
