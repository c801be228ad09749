#!/usr/bin/env python3
"""ResNet-50 convolutions at batch 256: the hand-written NHWC implicit GEMM
(csrc/hip/conv.hip) against MIOpen (F.conv2d / aten.convolution_backward,
bf16 channels_last) — forward, input gradient, weight gradient — and, for the
1×1 stride-1 shapes, against the token-major GEMMs ops.conv1x1 uses (gemm_nt /
gemm_dw); interleaved rounds in one process, median µs per call and TFLOP/s.

    python tools/conv_probe.py [--batch 256] [--iters 20] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (C, H, K, R, stride): every distinct 3×3 and strided 1×1 of ResNet-50 v1.5
SHAPES = [(64, 56, 64, 3, 1), (128, 56, 128, 3, 2), (128, 28, 128, 3, 1), (256, 28, 256, 3, 2),
          (256, 14, 256, 3, 1), (512, 14, 512, 3, 2), (512, 7, 512, 3, 1),
          (256, 56, 512, 1, 2), (512, 28, 1024, 1, 2), (1024, 14, 2048, 1, 2)]
# every distinct 1×1 stride-1 (conv1 / conv3 / layer1 downsample)
SHAPES_1X1 = [(64, 56, 64, 1, 1), (64, 56, 256, 1, 1), (256, 56, 64, 1, 1), (256, 56, 128, 1, 1),
              (128, 28, 512, 1, 1), (512, 28, 128, 1, 1), (512, 28, 256, 1, 1), (256, 14, 1024, 1, 1),
              (1024, 14, 256, 1, 1), (1024, 14, 512, 1, 1), (512, 7, 2048, 1, 1), (2048, 7, 512, 1, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only-1x1", action="store_true")
    a = ap.parse_args()
    import torch
    import torch.nn.functional as F
    from paddle_operator_amd import _native
    from paddle_operator_amd.utils.tuning import use_shipped_miopen_db
    use_shipped_miopen_db()
    m = _native.require_hip()
    torch.backends.cudnn.benchmark = False
    dev = torch.device("cuda", 0)
    cb = torch.ops.aten.convolution_backward

    def timeit(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3

    for C, H, K, R, st in ([] if a.only_1x1 else SHAPES) + SHAPES_1X1:
        N, pad = a.batch, (R - 1) // 2
        x = torch.randn(N, C, H, H, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(K, C, R, R, device=dev) / (C * R * R) ** 0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        y = F.conv2d(x, w, stride=st, padding=pad)
        dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
        wt = m.conv_weight_t(w)
        fl = 2.0 * y.numel() * C * R * R
        cand = {
            "hip_fwd": lambda: m.conv_fwd(x, w, st, pad, True),
            "miopen_fwd": lambda: F.conv2d(x, w, stride=st, padding=pad),
            "hip_dgrad": lambda: m.conv_dgrad(dy, wt, C, R, R, H, H, st, pad),
            "miopen_dgrad": lambda: cb(dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                       [True, False, False]),
            "hip_wgrad": lambda: m.conv_wgrad(dy, x, R, R, st, pad),
            "miopen_wgrad": lambda: cb(dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                       [False, True, False]),
        }
        if hasattr(m, "conv_wgrad_mode"):  # the 128 × 128 wgrad kernel where the gathered dw4 path would run
            def wg1():
                prev = m.conv_wgrad_mode(0)
                try:
                    return m.conv_wgrad(dy, x, R, R, st, pad)
                finally:
                    m.conv_wgrad_mode(prev)
            cand["hip1_wgrad"] = wg1
        if hasattr(m, "conv_wgrad_c64_mode") and C == K and C in (64, 128) and R == 3:
            def wg64off():
                prev = m.conv_wgrad_c64_mode(0)
                try:
                    return m.conv_wgrad(dy, x, R, R, st, pad)
                finally:
                    m.conv_wgrad_c64_mode(prev)
            cand["hip_pertap_wgrad"] = wg64off
        if R == 1 and st == 1:
            T = N * H * H
            x2, dy2, w2 = x.permute(0, 2, 3, 1).reshape(T, C), dy.permute(0, 2, 3, 1).reshape(T, K), w.view(K, C)
            w2t = w2.t().contiguous()
            gw = torch.empty(K, C, device=dev, dtype=torch.bfloat16)
            if m.gemm_nt_supported(T, K, C):
                cand["gemm_fwd"] = lambda: m.gemm_nt(x2, w2)
            if m.gemm_nt_supported(T, C, K):
                cand["gemm_dgrad"] = lambda: m.gemm_nt(dy2, w2t)
            if ((K + 255) // 256) * (C // 256) >= 8:
                cand["gemm_wgrad"] = lambda: m.gemm_dw(dy2, x2, gw, False)
        times = {k: [] for k in cand}
        for _ in range(a.rounds):
            for k, fn in cand.items():
                times[k].append(timeit(fn))
        rec = {"shape": f"{N}x{C}x{H}x{H} -> {K} r{R} s{st}"}
        for k, v in times.items():
            us = statistics.median(v)
            rec[k] = round(us, 1)
            rec[k + "_TF"] = round(fl / us / 1e6, 1)
        # numerics: the forward against fp32 on a corner of the batch
        ref = F.conv2d(x[:2].float(), w.float(), stride=st, padding=pad)
        got = m.conv_fwd(x[:2].contiguous(memory_format=torch.channels_last), w, st, pad, False)[0]
        rec["fwd_rel_err"] = round(((got.float() - ref).norm() / ref.norm()).item(), 5)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
