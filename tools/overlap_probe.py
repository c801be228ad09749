#!/usr/bin/env python3
"""How the step's kernels behave when a few CUs are held by another kernel —
the situation of an RCCL all-reduce kernel running on the overlap stream during
the backward at N > 1 (its workgroups hold their CUs until the transfer ends).

Each kernel is timed alone, then launched right after H side-stream kernels
that each hold one whole CU for ≈ ``--hold-us`` (a one-tile, one-slice
``gemm_dw``: one workgroup with 128 KiB of LDS and the full register file —
``torch.cuda._sleep``'s one-wave kernel leaves room beside a GEMM wave and
holds nothing).  A kernel whose grid is one resident round of long workgroups
(the persistent GEMMs, the split-K weight gradient, the one-round LayerNorm
backward) cannot start its workgroups on the held CUs until they free up, so it
ends at ≈ hold + its own time; a kernel with many short workgroups (attention)
loses ≈ H / 256 of its throughput.

    python tools/overlap_probe.py [--holds 1,3] [--hold-us 300] [--iters 10]

gemm_nt4 runs in both tile orders (static: one GPU; dynamic per-XCD counters:
the experiment switch gemm_nt4_dynamic(1); tools/overlap_step_probe.py
measures both inside the training step).
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--holds", default="1,3")
    ap.add_argument("--hold-us", type=float, default=300.0)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch
    from paddle_operator_amd import _native
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    T, C, H = 65536, 1024, 16
    bf = dict(device=dev, dtype=torch.bfloat16)
    a_dx = torch.randn(T, C, **bf)
    w_t = torch.randn(C, C, **bf) / 32
    dy4 = torch.randn(T, 4 * C, **bf)
    w1 = torch.randn(C, 4 * C, **bf) / 64
    x = torch.randn(T, C, **bf)
    dw = torch.empty(4 * C, C, **bf)
    lw, lb = torch.ones(C, **bf), torch.zeros(C, **bf)
    qkv = torch.randn(64, 1024, 3 * C, **bf)
    _, mean, rstd = m.layernorm_fwd(x, lw, lb, 1e-5)[:3]
    def nt4(order, fn):  # gemm_nt4 with its tile order: 0 static (the default), 1 dynamic
        def run_():
            prev = m.gemm_nt4_dynamic(order)
            try:
                return fn()
            finally:
                m.gemm_nt4_dynamic(prev)
        return run_

    kernels = {
        "gemm_nt4 proj dX [65536x1024, K 1024], static order": nt4(0, lambda: m.gemm_nt(a_dx, w_t)),
        "gemm_nt4 proj dX [65536x1024, K 1024], dynamic order": nt4(1, lambda: m.gemm_nt(a_dx, w_t)),
        "gemm_nt4 fc1 dX [65536x1024, K 4096], static order": nt4(0, lambda: m.gemm_nt(dy4, w1)),
        "gemm_nt4 fc1 dX [65536x1024, K 4096], dynamic order": nt4(1, lambda: m.gemm_nt(dy4, w1)),
        "gemm_dw4 fc1 dW [4096x1024, K 65536]": lambda: m.gemm_dw(dy4, x, dw, False),
        "layernorm_bwd [65536x1024]": lambda: m.layernorm_bwd(a_dx, x, lw, mean, rstd),
        "attn_fwd [B64 H16 S1024]": lambda: m.attn_fwd(qkv, H),
    }
    side = [torch.cuda.Stream(dev) for _ in range(4)]
    # the hog: one 256 x 256 output tile, one k-slice of Th tokens, sized to ≈ hold_us
    def hog_of(th):
        hy, hx = torch.randn(th, 256, **bf), torch.randn(th, 256, **bf)
        ho = torch.empty(256, 256, **bf)
        return lambda: m.gemm_dw(hy, hx, ho, False, 1)

    def once(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    th = 4096
    t4 = once(hog_of(th))
    th = max(128, int(th * a.hold_us / t4) // 128 * 128)
    hog = hog_of(th)
    print(json.dumps({"hog_tokens": th, "hog_us": round(once(hog), 1)}), flush=True)

    def run(fn, holds):
        ts = []
        for _ in range(a.iters):
            torch.cuda.synchronize()
            cur = torch.cuda.current_stream(dev)
            for s in side[:holds]:
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    hog()
            b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b0.record()
            fn()
            b1.record()
            torch.cuda.synchronize()
            ts.append(b0.elapsed_time(b1) * 1e3)
        return statistics.median(ts)

    holds = [int(h) for h in a.holds.split(",") if h]
    for name, fn in kernels.items():
        fn()
        rec = {"kernel": name, "alone_us": round(run(fn, 0), 1), "hold_us": a.hold_us}
        for h in holds:
            rec[f"held_{h}_cu_us"] = round(run(fn, h), 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
