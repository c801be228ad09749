"""gemm_nt mainloops A/B on the GPT-2-medium projection shapes: the 8-wave
ring (impl 0, gemm_nt.hip), the 4-wave 128×128-per-wave loop (impl 1,
gemm_nt4.hip) and hipBLASLt (tuned tables), interleaved rounds in one process
(median of --rounds × --iters).  Numerics: impl 1 must equal impl 0 bit for bit
(same k order), and impl 0 is checked against an fp32 reference on a slice.

    python tools/nt4_probe.py [--tokens 65536] [--iters 20] [--rounds 3] [--shapes qkv_fwd,fc2_fwd]
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
    ap.add_argument("--shapes", default="")
    ap.add_argument("--variants", type=int, default=1, help="gemm_nt4 schedule variants to A/B (impl 1..N)")
    ap.add_argument("--impls", default="", help="explicit impl list, e.g. 0,1,5,6 (first = reference)")
    a = ap.parse_args()
    enable_tuned_gemms()
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, C = a.tokens, 1024
    shapes = [("qkv_fwd", 3 * C, C, "bias"), ("proj_fwd", C, C, "plain"), ("fc1_fwd", 4 * C, C, "gelu"),
              ("fc2_fwd", C, 4 * C, "plain"), ("qkv_dx", C, 3 * C, "plain"), ("proj_dx", C, C, "plain"),
              ("fc1_dx", C, 4 * C, "plain"), ("fc2_dx", 4 * C, C, "dgelu"), ("lm_dx", C, 50304, "plain"),
              ("wide_plain", 4 * C, C, "plain"),  # fc1_fwd / fc2_dx GEMM without an epilogue
              ("fc1_gd", 4 * C, C, "gelu_gd"), ("fc2_dx_gd", 4 * C, C, "dgelu_gd")]  # the saved-GELU' pair
    if a.shapes:
        keep = set(a.shapes.split(","))
        shapes = [s for s in shapes if s[0] in keep]
    for name, N, K, epi in shapes:
        x = torch.empty(M, K, device=dev, dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
        w = torch.empty(N, K, device=dev, dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
        b = torch.empty(N, device=dev, dtype=torch.bfloat16).uniform_(-0.1, 0.1, generator=g)
        pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16).uniform_(-2, 2, generator=g)
        if epi in ("plain", "bias"):
            ours = (lambda: m.gemm_nt(x, w, b)) if epi == "bias" else (lambda: m.gemm_nt(x, w))
            lib = (lambda: F.linear(x, w, b)) if epi == "bias" else (lambda: F.linear(x, w))
        elif epi == "gelu":
            ours = lambda: m.gemm_nt_gelu(x, w, b)  # noqa: E731
            lib = lambda: m.bias_gelu_fwd(F.linear(x, w), b)  # noqa: E731
        elif epi == "gelu_gd":
            ours = lambda: m.gemm_nt_gelu(x, w, b, saved_grad=True)  # noqa: E731
            lib = lambda: m.bias_gelu_fwd(F.linear(x, w), b)  # noqa: E731
        elif epi == "dgelu_gd":
            ours = lambda: m.gemm_nt_dgelu(x, w, pre, b, saved_grad=True)  # noqa: E731
            lib = lambda: F.linear(x, w) * pre  # noqa: E731
        else:
            ours = lambda: m.gemm_nt_dgelu(x, w, pre, b)  # noqa: E731
            lib = lambda: m.bias_gelu_bwd(F.linear(x, w), pre, b)  # noqa: E731
        impls = [int(x) for x in a.impls.split(",")] if a.impls else [0] + [1 + v for v in range(a.variants)]
        outs = {}
        for impl in impls:
            m.gemm_nt_impl(impl)
            o = ours()
            outs[impl] = [t.clone() for t in (o if isinstance(o, (list, tuple)) else [o])]
        torch.cuda.synchronize()
        i0 = impls[0]
        ident = all(torch.equal(p, q) for i in impls[1:] for p, q in zip(outs[i0], outs[i]))
        maxdiff = max([(p.float() - q.float()).abs().max().item() for i in impls[1:] for p, q in zip(outs[i0], outs[i])] or [0.0])
        R = 512
        ref = x[-R:].float() @ w.float().t()
        c0 = outs[impls[-1]][0][-R:].float()
        if epi == "bias":
            ref = ref + b.float()
        ref_err = (c0 - ref).abs().max().item() if epi in ("plain", "bias", "gelu") else None
        del outs
        times = {f"nt{i}": [] for i in impls}
        times["lib"] = []
        for _ in range(a.rounds):
            for i in impls:
                m.gemm_nt_impl(i)
                times[f"nt{i}"].append(bench(ours, a.iters))
            times["lib"].append(bench(lib, a.iters))
        fl = 2.0 * M * N * K
        rec = {"shape": name, "N": N, "K": K, "epi": epi, "bitwise_equal": ident, "max_diff": maxdiff,
               "ref_err": ref_err}
        for k, v in times.items():
            med = statistics.median(v)
            rec[k + "_us"] = round(med, 1)
            rec[k + "_PF"] = round(fl / med / 1e9, 3)
        print(json.dumps(rec), flush=True)
        del x, w, b, pre


if __name__ == "__main__":
    main()
