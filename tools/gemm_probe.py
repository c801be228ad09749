"""GEMM microbenchmark for the GPT-2-medium training shapes (hipBLASLt / rocBLAS / split-K / pdo kernels).

    python tools/gemm_probe.py [--tokens 32768] [--libs hipblaslt,rocblas] [--pdo]
"""
import argparse
import json
import sys
import time

import torch


def bench(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--libs", default="hipblaslt,rocblas")
    ap.add_argument("--pdo", action="store_true")
    a = ap.parse_args()
    T = a.tokens
    dev = torch.device("cuda")
    d = torch.bfloat16
    shapes = [("qkv", 1024, 3072), ("proj", 1024, 1024), ("fc1", 1024, 4096), ("fc2", 4096, 1024)]
    out = []
    for lib in a.libs.split(","):
        torch.backends.cuda.preferred_blas_library(lib)
        for name, fin, fout in shapes:
            X = torch.randn(T, fin, device=dev, dtype=d)
            W = torch.randn(fout, fin, device=dev, dtype=d) * 0.02
            dY = torch.randn(T, fout, device=dev, dtype=d)
            fl = 2.0 * T * fin * fout
            r = {"lib": lib, "gemm": name, "T": T, "in": fin, "out": fout}
            r["fwd_us"] = bench(lambda: torch.mm(X, W.t()))
            r["dx_us"] = bench(lambda: torch.mm(dY, W))
            dW = torch.empty(fout, fin, device=dev, dtype=d)
            r["dw_us"] = bench(lambda: torch.mm(dY.t(), X, out=dW))
            for s in (2, 4, 8):
                dYs = dY.view(s, T // s, fout).transpose(1, 2)
                Xs = X.view(s, T // s, fin)
                r[f"dw_split{s}_us"] = bench(lambda: torch.sum(torch.bmm(dYs, Xs), 0, out=dW))
            for k in list(r):
                if k.endswith("_us"):
                    r[k.replace("_us", "_tf")] = round(fl / (r[k] * 1e-6) / 1e12, 1)
                    r[k] = round(r[k], 1)
            print(json.dumps(r), flush=True)
            out.append(r)
    if a.pdo:
        sys.path.insert(0, ".")
        from paddle_operator_amd import ops
        for name, fin, fout in shapes:
            X = torch.randn(T, fin, device=dev, dtype=d)
            W = torch.randn(fout, fin, device=dev, dtype=d) * 0.02
            dY = torch.randn(T, fout, device=dev, dtype=d)
            fl = 2.0 * T * fin * fout
            r = {"lib": "pdo", "gemm": name}
            if hasattr(ops, "gemm_dw"):
                dW = torch.empty(fout, fin, device=dev, dtype=d)
                r["dw_us"] = bench(lambda: ops.gemm_dw(dY, X, dW))
                r["dw_tf"] = round(fl / (r["dw_us"] * 1e-6) / 1e12, 1)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
