"""gemm_nt (csrc/hip/gemm_nt.hip) vs hipBLASLt (tuned TunableOp tables) on the
GPT-2-medium projection shapes, forward and input-gradient forms, with the
fused GELU / GELU' epilogues against the unfused GEMM + bias-GELU kernel pair.

    python tools/nt_probe.py [--tokens 65536] [--iters 20]

Prints one JSON line per shape: µs and PF/s for both, and the max abs error of
a 256-row slice against an fp32 reference.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402
from paddle_operator_amd.utils.tuning import enable_tuned_gemms  # noqa: E402


def bench(fn, iters, warm=5):
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


def gelu_ref(x):
    return F.gelu(x, approximate="tanh")


def gelu_grad_ref(x):
    x = x.detach().requires_grad_(True)
    (g,) = torch.autograd.grad(F.gelu(x, approximate="tanh").sum(), x)
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    enable_tuned_gemms()
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M = a.tokens
    C = 1024
    shapes = [  # (name, N, K, epilogue)
        ("qkv_fwd", 3 * C, C, "bias"), ("proj_fwd", C, C, "plain"), ("fc1_fwd", 4 * C, C, "gelu"),
        ("fc2_fwd", C, 4 * C, "plain"), ("qkv_dx", C, 3 * C, "plain"), ("proj_dx", C, C, "plain"),
        ("fc1_dx", C, 4 * C, "plain"), ("fc2_dx", 4 * C, C, "dgelu"),
    ]
    for name, N, K, epi in shapes:
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
        w = (torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.03)
        b = (torch.randn(N, device=dev, dtype=torch.bfloat16, generator=g) * 0.1)
        pre = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
        R = 256
        ref = x[:R].float() @ w.float().t()
        if epi == "plain":
            ours = lambda: m.gemm_nt(x, w)  # noqa: E731
            lib = lambda: F.linear(x, w)  # noqa: E731
            out = ours()[:R].float()
            err = (out - ref).abs().max().item()
        elif epi == "bias":
            ours = lambda: m.gemm_nt(x, w, b)  # noqa: E731
            lib = lambda: F.linear(x, w, b)  # noqa: E731
            err = (ours()[:R].float() - (ref + b.float())).abs().max().item()
        elif epi == "gelu":
            ours = lambda: m.gemm_nt_gelu(x, w, b)  # noqa: E731
            lib = lambda: m.bias_gelu_fwd(F.linear(x, w), b)  # noqa: E731
            p, y = ours()
            err = max((p[:R].float() - ref).abs().max().item(),
                      (y[:R].float() - gelu_ref(p[:R].float() + b.float())).abs().max().item())
        else:
            dbuf = torch.zeros(N, device=dev, dtype=torch.bfloat16)
            ours = lambda: m.gemm_nt_dgelu(x, w, pre, b)  # noqa: E731
            lib = lambda: m.bias_gelu_bwd(F.linear(x, w), pre, b)  # noqa: E731
            dx, db = ours()
            dyr = (x.float() @ w.float().t()).to(torch.bfloat16).float()
            dref = dyr * gelu_grad_ref(pre.float() + b.float())
            err = max((dx.float() - dref).abs().max().item() / max(dref.abs().max().item(), 1e-6),
                      (db.float() - dref.sum(0)).abs().max().item() / max(dref.sum(0).abs().max().item(), 1e-6))
            del dbuf, dyr, dref
        t_o = bench(ours, a.iters)
        t_l = bench(lib, a.iters)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "epi": epi, "nt_us": round(t_o, 1),
                          "lib_us": round(t_l, 1), "nt_PF": round(fl / t_o / 1e9, 3),
                          "lib_PF": round(fl / t_l / 1e9, 3), "speedup": round(t_l / t_o, 3),
                          "max_err": err}), flush=True)
        del x, w, b, pre


if __name__ == "__main__":
    main()
