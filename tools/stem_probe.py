"""ResNet-50 stem (7×7 / stride 2 / pad 3, 3 → 64 channels) at batch N: the
space-to-depth HIP kernels (stem_fwd = s2d + weight transform + implicit GEMM
with BatchNorm tile statistics; stem_wgrad = tap-group kernel + folds) against
MIOpen's forward and weight-gradient solvers on the same tensors.
    python tools/stem_probe.py [N] [iters]     (one JSON line per product)
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
IT = int(sys.argv[2]) if len(sys.argv) > 2 else 20
m = _native.require_hip()
x = torch.randn(N, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 3, 7, 7, device="cuda") / 147 ** 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
y, st, z = m.stem_fwd(x, w, True)
dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
out = torch.zeros(64, 3, 7, 7, device="cuda").contiguous(memory_format=torch.channels_last)


def timed(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(IT):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / IT


def miopen_wgrad():
    torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                        [False, True, False])


flop = 2.0 * N * 112 * 112 * 64 * 147
for name, fn in (("hip_fwd", lambda: m.stem_fwd(x, w, True)), ("miopen_fwd", lambda: F.conv2d(x, w, stride=2, padding=3)),
                 ("hip_wgrad", lambda: m.stem_wgrad(dy, z, out)), ("miopen_wgrad", miopen_wgrad)):
    us = timed(fn)
    print(json.dumps({"op": name, "N": N, "us": round(us, 1), "tflops": round(flop / us / 1e6, 1)}), flush=True)
ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
rel = ((y.float() - ref).norm() / ref.norm()).item()
print(json.dumps({"check": "fwd_rel", "value": rel}))
