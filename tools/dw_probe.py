"""Weight-gradient GEMM alternatives at the GPT-2-medium B=64 shapes (T = 65536 tokens).

Runs with TunableOp online tuning into a scratch file so every variant gets its
best hipBLASLt/rocBLAS solution, then times each variant (incl. the split-K
fold into the arena).  python tools/dw_probe.py [--tokens 65536]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=10, warm=2):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--shapes", default="qkv,proj,fc1,fc2,lm")
    ap.add_argument("--pdo-only", action="store_true", help="time the HIP dW GEMM against the shipped-table path")
    a = ap.parse_args()
    if a.pdo_only:
        return pdo_vs_lib(a)
    from paddle_operator_amd import _native
    m = _native.require_hip()
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.environ.get("PDO_TUNE_OUT", "/tmp/dw_probe_tune%d.csv"))
    tun.set_max_tuning_duration(int(os.environ.get("PDO_TUNE_MS", "60")))
    T = a.tokens
    dev = torch.device("cuda")
    table = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096), "lm": (50304, 1024)}
    for name in a.shapes.split(","):
        Fo, K = table[name]
        dy = torch.randn(T, Fo, device=dev).bfloat16()
        x = torch.randn(T, K, device=dev).bfloat16()
        g = torch.zeros(Fo, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * Fo * K
        res = {"gemm": name, "Fo": Fo, "K": K}
        for s in (1, 2, 4, 8):
            if s == 1:
                fn = lambda: g.addmm_(dy.t(), x)
            else:
                ws = torch.empty(s, Fo, K, device=dev, dtype=torch.bfloat16)
                dys = dy.view(s, T // s, Fo).transpose(1, 2)
                xs = x.view(s, T // s, K)

                def fn(dys=dys, xs=xs, ws=ws):
                    torch.bmm(dys, xs, out=ws)
                    m.splitk_add(ws, g, True)
            res[f"a_s{s}_us"] = round(bench(fn), 1)
        # swapped orientation: dWᵀ = Xᵀ·dY, then a transpose into the arena
        gt = torch.empty(K, Fo, device=dev, dtype=torch.bfloat16)
        for s in (1, 2, 4):
            if s == 1:
                fn = lambda: (torch.mm(x.t(), dy, out=gt), m.transpose(gt))
            else:
                ws = torch.empty(s, K, Fo, device=dev, dtype=torch.bfloat16)
                xs = x.view(s, T // s, K).transpose(1, 2)
                dys = dy.view(s, T // s, Fo)

                def fn(dys=dys, xs=xs, ws=ws):
                    torch.bmm(xs, dys, out=ws)
                    m.splitk_add(ws, gt, False)
                    m.transpose(gt)
            res[f"b_s{s}_us"] = round(bench(fn), 1)
        best = min((v, k) for k, v in res.items() if k.endswith("_us"))
        res["best"] = best[1]
        res["best_tf"] = round(fl / (best[0] * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)


def pdo_vs_lib(a):
    from paddle_operator_amd import _native, ops
    from paddle_operator_amd.utils.tuning import enable_tuned_gemms
    m = _native.require_hip()
    enable_tuned_gemms()
    T = a.tokens
    dev = torch.device("cuda")
    table = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096), "lm": (50304, 1024)}
    for name in a.shapes.split(","):
        Fo, K = table[name]
        g = torch.Generator(device=dev).manual_seed(0)
        dy = (0.01 * torch.randn(T, Fo, device=dev, generator=g)).bfloat16()
        x = torch.randn(T, K, device=dev, generator=g).bfloat16()
        w = torch.zeros(Fo, K, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * Fo * K
        res = {"gemm": name, "splits": m.gemm_dw_splits(T, Fo, K)}
        gl = torch.zeros(Fo, K, device=dev, dtype=torch.bfloat16)

        class P:  # stand-in parameter with an arena-style grad
            pass
        p = P()
        p.grad = gl
        p._pdo_direct = True
        p._pdo_ready = lambda _p: None
        variants = [int(v) for v in os.environ.get("DW_SPLITS", "0").split(",")]
        lib, pdo = [], {v: [] for v in variants}
        for _ in range(5):
            lib.append(bench(lambda: ops._weight_grad_lib(p, dy, x)))
            if res["splits"]:
                for v in variants:
                    pdo[v].append(bench(lambda: m.gemm_dw(dy, x, w, True, v)))
        res["lib_us"] = round(sorted(lib)[2], 1)
        res["lib_tf"] = round(fl / (res["lib_us"] * 1e-6) / 1e12, 1)
        if res["splits"]:
            for v in variants:
                t = sorted(pdo[v])[2]
                res[f"pdo{v}_us"] = round(t, 1)
                res[f"pdo{v}_tf"] = round(fl / (t * 1e-6) / 1e12, 1)
            w.zero_()
            gl.zero_()
            m.gemm_dw(dy, x, w, True)
            ops._weight_grad_lib(p, dy, x)
            res["maxdiff_rel"] = ((w.float() - gl.float()).abs().max() / gl.float().abs().max()).item()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
