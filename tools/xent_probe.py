#!/usr/bin/env python3
"""Fused LM-head cross-entropy pass (csrc/hip/xent.hip xent_fused) at the GPT-2-medium
shape: µs per call and achieved TB/s (the logits read, dlogits written in place).

    python tools/xent_probe.py [--tokens 65536] [--vocab 50257] [--vp 50304]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--vp", type=int, default=50304)
    a = ap.parse_args()
    import torch

    from paddle_operator_amd import _native
    from tools.attn_probe import bench
    m = _native.require_hip()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    base = (3 * torch.randn(a.tokens, a.vp, device=dev, generator=g)).bfloat16()
    tgt = torch.randint(0, a.vocab, (a.tokens,), device=dev, generator=g)
    inv = torch.full((1,), 1.0 / a.tokens, device=dev)
    lg = base.clone()
    loss = m.xent_fused(lg, tgt, inv, a.vocab)
    # reference on a slice: fp32 softmax − onehot
    R = 64
    x = base[:R, :a.vocab].float()
    p = torch.softmax(x, dim=1)
    p[torch.arange(R, device=dev), tgt[:R]] -= 1.0
    err = float((lg[:R, :a.vocab].float() - p / a.tokens).abs().max() * a.tokens)
    ref_loss = float(torch.nn.functional.cross_entropy(base[:, :a.vocab].float()[:4096], tgt[:4096]))
    t = sorted(bench(lambda: m.xent_fused(lg, tgt, inv, a.vocab), iters=5, warm=1) for _ in range(3))[1]
    print(json.dumps({"us": round(t, 1),
                      "TBps": round(2 * a.tokens * a.vp * 2 / t / 1e6, 2), "dlogit_err_x_count": err,
                      "loss": float(loss), "ref_loss_first4096": ref_loss}))


if __name__ == "__main__":
    main()
