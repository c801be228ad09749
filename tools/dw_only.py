"""Minimal driver for PMC passes: gemm_dw (HIP) and hipBLASLt dYᵀ·X on one GPT-2 dW shape.
    python tools/dw_only.py [M] [N] [iters] [impl]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402
from paddle_operator_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
it = int(sys.argv[3]) if len(sys.argv) > 3 else 3
impl = int(sys.argv[4]) if len(sys.argv) > 4 else -1
enable_tuned_gemms()
m = _native.require_hip()
if impl >= 0:
    m.gemm_dw_impl(impl)
T = 65536
dy = torch.randn(T, M, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    m.gemm_dw(dy, x, out, False)
    torch.mm(dy.t(), x, out=out)
torch.cuda.synchronize()
