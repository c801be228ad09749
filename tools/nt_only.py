"""Minimal driver for PMC passes: gemm_nt and hipBLASLt on one GPT-2 shape.
    python tools/nt_only.py [N] [K] [iters] [impl] [gelu]
With a 5th argument "gelu", each iteration also runs the fused bias-GELU
epilogue form (gemm_nt_gelu) and the fused GELU'-dX form (gemm_nt_dgelu) of the
same shape, for per-epilogue counter comparisons."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402
from paddle_operator_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
it = int(sys.argv[3]) if len(sys.argv) > 3 else 5
impl = int(sys.argv[4]) if len(sys.argv) > 4 else -1
enable_tuned_gemms()
m = _native.require_hip()
if impl >= 0:
    m.gemm_nt_impl(impl)
x = torch.randn(65536, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
gelu = len(sys.argv) > 5 and sys.argv[5] == "gelu"
b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
pre = torch.randn(65536, N, device="cuda", dtype=torch.bfloat16)
for _ in range(it):
    m.gemm_nt(x, w)
    if gelu:
        m.gemm_nt_gelu(x, w, b)
        m.gemm_nt_dgelu(x, w, pre, b)
    else:
        F.linear(x, w)
torch.cuda.synchronize()
