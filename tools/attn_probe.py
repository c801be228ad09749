"""Causal attention microbenchmark (GPT-2-medium shape) — pdo HIP kernels vs torch SDPA.

    python tools/attn_probe.py [--B 32] [--S 1024] [--H 16]
"""
import argparse
import os
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20, warm=5):
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
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--H", type=int, default=16)
    a = ap.parse_args()
    from paddle_operator_amd import _native
    m = _native.require_hip()
    B, S, H, D = a.B, a.S, a.H, 64
    dev = torch.device("cuda")
    qkv = torch.randn(B, S, 3, H, D, device=dev, dtype=torch.bfloat16)
    dout = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16)
    scale = D ** -0.5
    flops_fwd = 2 * 2 * B * H * S * S * D / 2  # causal: half of QK^T and PV
    res = {"B": B, "S": S, "H": H}

    o, lse = m.attn_fwd(qkv.view(B, S, 3 * H * D), H)
    res["pdo_fwd_us"] = bench(lambda: m.attn_fwd(qkv.view(B, S, 3 * H * D), H))
    res["pdo_bwd_us"] = bench(lambda: m.attn_bwd(dout.view(B, S, H * D), qkv.view(B, S, 3 * H * D), o, lse, H))
    # correctness vs SDPA (fp32 math on bf16 inputs)
    q, k, v = [qkv[:, :, i].transpose(1, 2) for i in range(3)]
    ref = F.scaled_dot_product_attention(q.float(), k.float(), v.float(), is_causal=True)
    err = (o.view(B, S, H, D).transpose(1, 2).float() - ref).abs().max().item()
    res["fwd_max_abs_err"] = err
    qq, kk, vv = [x.detach().clone().requires_grad_(True) for x in (q, k, v)]
    res["sdpa_fwd_us"] = bench(lambda: F.scaled_dot_product_attention(qq, kk, vv, is_causal=True))
    y = F.scaled_dot_product_attention(qq, kk, vv, is_causal=True)
    g = dout.transpose(1, 2)
    res["sdpa_bwd_us"] = bench(lambda: torch.autograd.grad(y, (qq, kk, vv), g, retain_graph=True))
    for k_ in ("pdo_fwd", "sdpa_fwd"):
        res[k_ + "_tf"] = round(flops_fwd / (res[k_ + "_us"] * 1e-6) / 1e12, 1)
    for k_ in ("pdo_bwd", "sdpa_bwd"):
        res[k_ + "_tf"] = round(2.5 * flops_fwd / (res[k_ + "_us"] * 1e-6) / 1e12, 1)
    print(json.dumps({k_: (round(v_, 1) if isinstance(v_, float) and "err" not in k_ else v_) for k_, v_ in res.items()}))


if __name__ == "__main__":
    main()
