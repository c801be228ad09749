"""ResNet-50's 1×1 stride-1 convolutions (batch 256, bf16, channels_last): MIOpen
(F.conv2d + aten.convolution_backward per gradient) against the same products
as token-major GEMMs — forward y = x·Wᵀ and input gradient dX = dY·W on
gemm_nt4 where its contract holds (else hipBLASLt), weight gradient dW = dYᵀ·X
on gemm_dw4 where its contract holds (else hipBLASLt over token slices + fold).
Per shape µs (median of --iters after warm-up) and the per-step sum weighted by
how often ResNet-50 uses the shape.

    python tools/conv1x1_probe.py [--batch 256] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native, ops  # noqa: E402

# (Cin, Cout, H, uses per step): conv1 / conv3 / stride-1 downsample of the bottlenecks
SHAPES = [
    (64, 64, 56, 1), (256, 64, 56, 2), (64, 256, 56, 4),
    (256, 128, 56, 1), (512, 128, 28, 3), (128, 512, 28, 4),
    (512, 256, 28, 1), (1024, 256, 14, 5), (256, 1024, 14, 6),
    (1024, 512, 14, 1), (2048, 512, 7, 2), (512, 2048, 7, 3),
]


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    m = _native.require_hip()
    dev = torch.device("cuda")
    tot = {"miopen": 0.0, "gemm": 0.0}
    for cin, cout, h, uses in SHAPES:
        g = torch.Generator(device=dev).manual_seed(cin + cout + h)
        x = torch.randn(a.batch, cin, h, h, device=dev, generator=g, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (0.05 * torch.randn(cout, cin, 1, 1, device=dev, generator=g)).to(torch.bfloat16)
        dy = torch.randn(a.batch, cout, h, h, device=dev, generator=g, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        cb = torch.ops.aten.convolution_backward
        mi = {
            "fwd": timed(lambda: F.conv2d(x, w), a.iters),
            "dx": timed(lambda: cb(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]), a.iters),
            "dw": timed(lambda: cb(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]), a.iters),
        }
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        w2 = w.view(cout, cin)
        wt = w2.t().contiguous()
        T = x2.shape[0]
        nt_f = bool(m.gemm_nt_supported(T, cout, cin))
        nt_d = bool(m.gemm_nt_supported(T, cin, cout))
        g_out = torch.empty(cout, cin, device=dev, dtype=torch.bfloat16)
        dw_hip = bool(m.gemm_dw_splits(T, cout, cin)) if hasattr(m, "gemm_dw_splits") else False

        def dwf():
            if not m.gemm_dw(dy2, x2, g_out, False):
                s = 64
                while T % s:
                    s //= 2
                part = torch.bmm(dy2.view(s, T // s, cout).transpose(1, 2), x2.view(s, T // s, cin))
                g_out.copy_(part.sum(0, dtype=torch.float32))
        def dw_bmm():
            part = torch.bmm(dy2.view(64, T // 64, cout).transpose(1, 2), x2.view(64, T // 64, cin))
            g_out.copy_(part.sum(0, dtype=torch.float32))
        ge = {
            "fwd": timed(lambda: m.gemm_nt(x2, w2) if nt_f else F.linear(x2, w2), a.iters),
            "dx": timed(lambda: m.gemm_nt(dy2, wt) if nt_d else F.linear(dy2, wt), a.iters),
            "dw": timed(dwf, a.iters),
            "dw_bmm64": timed(dw_bmm, a.iters),
        }
        # numerics of the GEMM path's weight gradient against MIOpen's
        dwf()
        ref = cb(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])[1].view(cout, cin)
        err = ((g_out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        rec = {"cin": cin, "cout": cout, "h": h, "uses": uses, "miopen_us": {k: round(v, 1) for k, v in mi.items()},
               "gemm_us": {k: round(v, 1) for k, v in ge.items()}, "nt_fwd": nt_f, "nt_dx": nt_d,
               "dw_rel_err": round(err, 4)}
        print(json.dumps(rec), flush=True)
        tot["miopen"] += uses * sum(mi.values())
        tot["gemm"] += uses * (min(mi["fwd"], ge["fwd"]) + min(mi["dx"], ge["dx"])
                               + min(mi["dw"], ge["dw"], ge["dw_bmm64"]))
    print(json.dumps({"per_step_ms": {k: round(v / 1e3, 3) for k, v in tot.items()},
                      "note": "gemm = per product the faster of the two"}), flush=True)


if __name__ == "__main__":
    main()
