"""LM-head weight gradient on 1×MI355X: the shipped path for the 50304-row
vocabulary (4-slice batched hipBLASLt GEMM + HIP fold) against the HIP
gemm_dw kernel on a 256-multiple vocabulary pad (50432), per split count.

    python tools/lm_dw_probe.py
"""
import json
import sys

import torch

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.attn_probe import bench  # noqa: E402
from paddle_operator_amd import _native  # noqa: E402

m = _native.require_hip()
T, C = 65536, 1024
d = torch.device("cuda")
x = torch.randn(T, C, device=d, dtype=torch.bfloat16)
out = {}
for V in (50304, 50432):
    dy = torch.randn(T, V, device=d, dtype=torch.bfloat16) * 0.01
    g = torch.zeros(V, C, device=d, dtype=torch.bfloat16)
    s = 4
    part = torch.empty(s, V, C, device=d, dtype=torch.bfloat16)

    def lib():
        torch.bmm(dy.view(s, T // s, V).transpose(1, 2), x.view(s, T // s, C), out=part)
        m.splitk_add(part, g, True)

    out[f"lib_split4_V{V}"] = bench(lib, iters=5, warm=2)
    if V % 128 == 0:
        ref = (dy.float().t() @ x.float())
        out[f"gemm_dw_auto_splits_V{V}"] = m.gemm_dw_splits(T, V, C)
        for sp in (0, 1, 2, 4, 8):
            g.zero_()
            assert m.gemm_dw(dy, x, g, False, sp)
            err = ((g.float() - ref).abs().max() / ref.abs().max()).item()
            out[f"gemm_dw_s{sp}_V{V}"] = bench(lambda: m.gemm_dw(dy, x, g, True, sp), iters=5, warm=2)
            out[f"gemm_dw_s{sp}_relerr"] = err
        del ref
    del dy, part, g
    torch.cuda.empty_cache()
res = {}
for k, v in out.items():
    if k.endswith("relerr"):
        res[k] = round(v, 5)
    elif "auto" in k:
        res[k] = v
    else:
        V = int(k.rsplit("V", 1)[1])
        res[k] = (round(v, 1), round(2 * T * V * C / (v * 1e-6) / 1e12))
print(json.dumps(res))
