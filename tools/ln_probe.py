#!/usr/bin/env python3
"""LayerNorm kernels at the GPT-2-medium step's shape (65536 × 1024 bf16):
forward, backward, and the backward with the residual gradient joined and the
folded bias's column sum (the step's ``ln_bwd_kernel<2, true, 3>``); µs per
call (median of rounds) and the HBM bytes each moves per µs.

    python tools/ln_probe.py [--rows 65536] [--cols 1024] [--iters 20] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--cols", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from paddle_operator_amd import _native
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    bf = dict(device=dev, dtype=torch.bfloat16)
    N, C = a.rows, a.cols
    x, dy, dres = (torch.randn(N, C, **bf) for _ in range(3))
    w, b = torch.randn(C, **bf), torch.randn(C, **bf)
    _, mean, rstd = m.layernorm_fwd(x, w, b, 1e-5)
    e = 2 * N * C  # bytes of one [N, C] bf16 tensor
    cases = {
        "ln_fwd": (lambda: m.layernorm_fwd(x, w, b, 1e-5), 2 * e),
        "ln_bwd": (lambda: m.layernorm_bwd(dy, x, w, mean, rstd), 3 * e),
        "ln_bwd_add_rbias": (lambda: m.layernorm_bwd_add(dy, x, w, mean, rstd, dres, True), 4 * e),
    }

    def timeit(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3

    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (fn, _) in cases.items():
            res[k].append(timeit(fn))
    for k, (_, nbytes) in cases.items():
        us = statistics.median(res[k])
        print(json.dumps({"kernel": k, "rows": N, "cols": C, "us": round(us, 1), "TB_per_s": round(nbytes / us / 1e6, 2)}))


if __name__ == "__main__":
    main()
