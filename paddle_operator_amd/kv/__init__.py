"""paddle_operator_amd.kv"""
