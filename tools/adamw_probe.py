#!/usr/bin/env python3
"""Fused AdamW over a GPT-2-medium-sized arena: the kernel variants of
csrc/hip/optim.hip (set_adamw_variant), interleaved, with achieved TB/s
(28 B per element: bf16 grad + fp32 master/m/v read, the same written back
+ the bf16 parameter) and the largest parameter difference to variant 1.

    python tools/adamw_probe.py [--n 406847488] [--variants 1,2,3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=355 * 2 ** 20)
    ap.add_argument("--variants", default="1,2,3")
    a = ap.parse_args()
    import torch

    from paddle_operator_amd import _native
    from tools.attn_probe import bench
    m = _native.require_hip()
    dev = torch.device("cuda")
    n = a.n // 1024 * 1024
    gen = torch.Generator(device=dev).manual_seed(0)
    g = (1e-2 * torch.randn(n, device=dev, generator=gen)).bfloat16()
    master0 = torch.randn(n, device=dev, generator=gen)
    m10 = 1e-3 * torch.randn(n, device=dev, generator=gen)
    m20 = 1e-6 * torch.rand(n, device=dev, generator=gen)
    decay = torch.ones(n // 1024, device=dev)
    norm = torch.tensor([4.0, 0.0], device=dev)
    vs = [int(v) for v in a.variants.split(",")]
    outs = {}
    for v in vs:  # one step from the same state: numerics
        m.set_adamw_variant(v)
        p = torch.empty(n, device=dev, dtype=torch.bfloat16)
        w, m1, m2 = master0.clone(), m10.clone(), m20.clone()
        m.adamw_flat(p, g, w, m1, m2, decay, norm, 3e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.0975, 0.5, 1.0)
        outs[v] = w
    ts = {v: [] for v in vs}
    p = torch.empty(n, device=dev, dtype=torch.bfloat16)
    w, m1, m2 = master0.clone(), m10.clone(), m20.clone()
    for _ in range(5):
        for v in vs:
            m.set_adamw_variant(v)
            ts[v].append(bench(lambda: m.adamw_flat(p, g, w, m1, m2, decay, norm, 3e-4, 0.9, 0.95, 1e-8, 0.1, 0.1,
                                                    0.0975, 0.5, 1.0), iters=10, warm=2))
    for v in vs:
        t = sorted(ts[v])[2]
        d = float(((outs[v] - outs[vs[0]]).abs() / (outs[vs[0]].abs() + 1e-3)).max())
        print(json.dumps({"variant": v, "us": round(t, 1), "TBps": round(28 * n / t / 1e6, 2),
                          "max_rel_diff_vs_first": d}))


if __name__ == "__main__":
    main()
