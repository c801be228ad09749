"""gemm_pnt (persistent, csrc/hip/gemm_pnt.hip) vs gemm_nt vs hipBLASLt (tuned
TunableOp tables) on the GPT-2-medium NT shapes, interleaved rounds in one
process (methodology: median over rounds).

    python tools/pnt_probe.py [--tokens 65536] [--iters 20] [--rounds 3]

One JSON line per shape: µs and PF/s of each variant.
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402
from paddle_operator_amd.utils.tuning import enable_tuned_gemms  # noqa: E402


def bench(fn, iters, warm=3):
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--grids", default="256")
    a = ap.parse_args()
    enable_tuned_gemms()
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, C = a.tokens, 1024
    shapes = [  # (name, N, K, epilogue)
        ("qkv_fwd", 3 * C, C, "bias"), ("proj_fwd", C, C, "plain"), ("fc1_fwd", 4 * C, C, "gelu"),
        ("fc2_dx", 4 * C, C, "dgelu"), ("proj_dx", C, C, "plain"), ("fc2_fwd", C, 4 * C, "plain"),
        ("qkv_dx", C, 3 * C, "plain"),
    ]
    grids = [int(x) for x in a.grids.split(",")]
    for name, N, K, epi in shapes:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.03
        b = torch.randn(N, device=dev, dtype=torch.bfloat16, generator=g) * 0.1
        pre = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
        var = {}
        if epi == "plain":
            var["lib"] = lambda: F.linear(x, w)  # noqa: E731
            var["nt"] = lambda: m.gemm_nt(x, w)  # noqa: E731
            for gr in grids:
                var[f"pnt{gr}"] = lambda gr=gr: m.gemm_pnt(x, w, 0, grid=gr)
            check = (m.gemm_pnt(x, w, 0)[0], m.gemm_nt(x, w))
        elif epi == "bias":
            var["lib"] = lambda: F.linear(x, w, b)  # noqa: E731
            var["nt"] = lambda: m.gemm_nt(x, w, b)  # noqa: E731
            for gr in grids:
                var[f"pnt{gr}"] = lambda gr=gr: m.gemm_pnt(x, w, 1, bias=b, grid=gr)
            check = (m.gemm_pnt(x, w, 1, bias=b)[0], m.gemm_nt(x, w, b))
        elif epi == "gelu":
            var["lib"] = lambda: m.bias_gelu_fwd(F.linear(x, w), b)  # noqa: E731
            var["nt"] = lambda: m.gemm_nt_gelu(x, w, b)  # noqa: E731
            for gr in grids:
                var[f"pnt{gr}"] = lambda gr=gr: m.gemm_pnt(x, w, 2, bias=b, grid=gr)
            check = (m.gemm_pnt(x, w, 2, bias=b)[1], m.gemm_nt_gelu(x, w, b)[1])
        else:
            var["lib"] = lambda: m.bias_gelu_bwd(F.linear(x, w), pre, b)  # noqa: E731
            var["nt"] = lambda: m.gemm_nt_dgelu(x, w, pre, b)  # noqa: E731
            for gr in grids:
                var[f"pnt{gr}"] = lambda gr=gr: m.gemm_pnt(x, w, 3, bias=b, pre=pre, grid=gr)
            check = (m.gemm_pnt(x, w, 3, bias=b, pre=pre)[0], m.gemm_nt_dgelu(x, w, pre, b)[0])
        same = bool(torch.equal(check[0], check[1]))
        times = {k: [] for k in var}
        for _ in range(a.rounds):
            for k, fn in var.items():
                times[k].append(bench(fn, a.iters))
        fl = 2.0 * M * N * K
        rec = {"shape": name, "M": M, "N": N, "K": K, "epi": epi, "pnt_equals_nt": same}
        for k, ts in times.items():
            t = statistics.median(ts)
            rec[f"{k}_us"] = round(t, 1)
            rec[f"{k}_PF"] = round(fl / t / 1e9, 3)
        print(json.dumps(rec), flush=True)
        del x, w, b, pre


if __name__ == "__main__":
    main()
