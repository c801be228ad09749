#!/usr/bin/env python3
"""GPT-2-medium GEMM shapes on the extension's default mainloops, one line of
µs per shape — for A/B of two builds of _pdo_hip.so on one box
(tools/gpu.sh 'soab:gemm_ab.py'): uses only functions every build exports."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from paddle_operator_amd import _native
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    T, C = 65536, 1024
    g = torch.Generator(device=dev).manual_seed(0)

    def r(*s):
        return (torch.randn(*s, device=dev, generator=g) * 0.05).bfloat16()

    x, w_qkv, w_fc1, w_fc2, w_lm = r(T, C), r(3 * C, C), r(4 * C, C), r(C, 4 * C), r(50304, C)
    h4, b4, pre = r(T, 4 * C), r(4 * C), r(T, 4 * C)
    dy, dq = r(T, C), r(T, 3 * C)
    gq = torch.empty(3 * C, C, device=dev, dtype=torch.bfloat16)
    g1 = torch.empty(4 * C, C, device=dev, dtype=torch.bfloat16)
    cases = {
        "qkv_fwd": lambda: m.gemm_nt(x, w_qkv),
        "fc1_gelu": lambda: m.gemm_nt_gelu(x, w_fc1, b4),
        "fc2_fwd": lambda: m.gemm_nt(h4, w_fc2),
        "fc2_dx_dgelu": lambda: m.gemm_nt_dgelu(dy, w_fc1, pre, b4),
        "lm_fwd": lambda: m.gemm_nt(x[:16384], w_lm),
        "dw_qkv": lambda: m.gemm_dw(dq, x, gq, False),
        "dw_fc1": lambda: m.gemm_dw(h4, x, g1, False),
    }
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    for name, fn in cases.items():
        fn()
        ts = []
        for _ in range(3):
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        out[name] = round(statistics.median(ts), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
