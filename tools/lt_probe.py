"""Probe hipBLASLt fused-epilogue support for the GPT-2 MLP shapes."""
import os
import sys
import torch
sys.path.insert(0, ".")
from paddle_operator_amd import _native

m = _native.require_hip()
E = {"GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160, "GELU_AUX_BIAS": 164, "DGELU": 192, "DGELU_BGRAD": 208, "BIAS": 4,
     "DEFAULT": 1}
cases = []
for T in (2048, 32768):
    # fc1 fwd: m=4096 n=T k=1024, ta=1 tb=0
    for name in ("DEFAULT", "BIAS", "GELU", "GELU_BIAS", "GELU_AUX", "GELU_AUX_BIAS"):
        for bf in (False, True):
            cases.append((name, 1, 0, 4096, T, 1024, "BIAS" in name, "AUX" in name, bf))
    for name in ("DGELU", "DGELU_BGRAD"):
        for bf in (False, True):
            cases.append((name, 0, 0, 4096, T, 1024, "BGRAD" in name, True, bf))
for c in cases:
    rc, msg = m.lt_probe(E[c[0]], *c[1:])
    print(c, rc, msg, flush=True)
