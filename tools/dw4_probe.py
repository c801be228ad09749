"""gemm_dw mainloops A/B on the GPT-2-medium weight-gradient shapes (T = 65536
tokens): the 8-wave ping-pong (impl 0, gemm_dw.hip), the 4-wave loop
(impl 1.., gemm_dw4.hip variants) and hipBLASLt (dYᵀ·X, tuned tables);
interleaved rounds in one process, median.  Numerics: every impl against an
fp32 reference on a 256 × 256 corner (split-K folds differ between impls, so
outputs are compared to the reference, not bitwise to each other).

    python tools/dw4_probe.py [--variants 2] [--rounds 3] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402
from paddle_operator_amd.utils.tuning import enable_tuned_gemms  # noqa: E402


def bench(fn, iters, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--variants", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    enable_tuned_gemms()
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    T, C = a.tokens, 1024
    shapes = [("qkv", 3 * C, C), ("proj", C, C), ("fc1", 4 * C, C), ("fc2", C, 4 * C)]
    impls = [0] + [1 + v for v in range(a.variants)]
    for name, M, N in shapes:
        dy = torch.empty(T, M, device=dev, dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
        x = torch.empty(T, N, device=dev, dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = dy[:, :256].float().t() @ x[:, :256].float()
        rec = {"shape": name, "M": M, "N": N, "T": T}
        for i in impls:
            m.gemm_dw_impl(i)
            rec[f"splits{i}"] = m.gemm_dw_splits(T, M, N)
            m.gemm_dw(dy, x, out, False)
            torch.cuda.synchronize()
            rec[f"err{i}"] = round((out[:256, :256].float() - ref).abs().max().item() / ref.abs().max().item(), 5)
        times = {f"dw{i}": [] for i in impls}
        times["lib"] = []
        for _ in range(a.rounds):
            for i in impls:
                m.gemm_dw_impl(i)
                times[f"dw{i}"].append(bench(lambda: m.gemm_dw(dy, x, out, False), a.iters))
            times["lib"].append(bench(lambda: torch.mm(dy.t(), x, out=out), a.iters))
        fl = 2.0 * T * M * N
        for k, v in times.items():
            med = statistics.median(v)
            rec[k + "_us"] = round(med, 1)
            rec[k + "_PF"] = round(fl / med / 1e9, 3)
        print(json.dumps(rec), flush=True)
        del dy, x, out
    m.gemm_dw_impl(1)


if __name__ == "__main__":
    main()
