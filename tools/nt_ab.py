"""gemm_nt vs hipBLASLt on one shape, back-to-back launches vs launches
separated by a device synchronize (where the two differ, the gap is a
sustained-load effect — clock or L2/MALL state — not the single-kernel time).

    python tools/nt_ab.py [--n 4096] [--k 1024] [--impls 1,6] [--iters 20] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_operator_amd import _native  # noqa: E402
from paddle_operator_amd.utils.tuning import enable_tuned_gemms  # noqa: E402


def timed(fn, iters, sync_each):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    if not sync_each:
        e[0].record()
        for _ in range(iters):
            fn()
        e[1].record()
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) / iters * 1e3
    ts = []
    for i in range(iters):
        e[2 * i].record()
        fn()
        e[2 * i + 1].record()
        torch.cuda.synchronize()
        time.sleep(0.002)
        ts.append(e[2 * i].elapsed_time(e[2 * i + 1]) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--impls", default="1,6")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    enable_tuned_gemms()
    m = _native.require_hip()
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.empty(a.m, a.k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    w = torch.empty(a.n, a.k, device="cuda", dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
    out = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
    fns = {}
    for i in [int(v) for v in a.impls.split(",")]:
        def f(i=i):
            m.gemm_nt_impl(i)
            return m.gemm_nt(x, w)
        fns[f"nt{i}"] = f
    fns["lib"] = lambda: torch.mm(x, w.t(), out=out)
    res = {k: {"b2b": [], "sync": []} for k in fns}
    for _ in range(a.rounds):
        for k, f in fns.items():
            res[k]["b2b"].append(timed(f, a.iters, False))
            res[k]["sync"].append(timed(f, a.iters, True))
    fl = 2.0 * a.m * a.n * a.k
    rec = {"M": a.m, "N": a.n, "K": a.k}
    for k, v in res.items():
        for mode, ts in v.items():
            us = statistics.median(ts)
            rec[f"{k}_{mode}_us"] = round(us, 1)
            rec[f"{k}_{mode}_PF"] = round(fl / us / 1e9, 3)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
