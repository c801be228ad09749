"""Minimal driver for PMC passes over the NHWC implicit-GEMM convolution:
one ResNet-50 shape, forward (+ BN tile stats) and input gradient, next to the
same-size token-major GEMM (gemm_nt) for a per-FLOP comparison.
    python tools/conv_only.py [C] [H] [K] [R] [stride] [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402

C, H, K, R, st, it = (int(v) for v in (sys.argv[1:7] + ["256", "14", "256", "3", "1", "5"][len(sys.argv) - 1:]))
N, pad = 256, (R - 1) // 2
m = _native.require_hip()
x = torch.randn(N, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).bfloat16().contiguous(
    memory_format=torch.channels_last)
y, _ = m.conv_fwd(x, w, st, pad, True)
dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
wt = m.conv_weight_t(w)
T = y.shape[0] * y.shape[2] * y.shape[3]
a = torch.randn(T, C * R * R, device="cuda", dtype=torch.bfloat16)
b = torch.randn(K, C * R * R, device="cuda", dtype=torch.bfloat16)
gemm = T % 256 == 0 and m.gemm_nt_supported(T, K, C * R * R)
for _ in range(it):
    m.conv_fwd(x, w, st, pad, True)
    m.conv_dgrad(dy, wt, C, R, R, H, H, st, pad)
    if gemm:
        m.gemm_nt(a, b)
torch.cuda.synchronize()
print("ok", T, gemm)
