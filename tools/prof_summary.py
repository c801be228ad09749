#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace`` database (ROCm 7.2 rocpd sqlite).

usage: python tools/prof_summary.py gpurun_out/prof/run_results.db [--steps K] [--top N]

Groups dispatches by kernel name (long Tensile names shortened), prints total
ms, calls, mean µs and share; with ``--steps`` also per-step ms.  Output is
plain markdown so it can be committed under ``profiles/``.
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    if name.startswith("Cijk_"):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        kind = name.split("_")[1] + "_" + name.split("_")[2]
        return f"hipBLASLt GEMM {kind} MT{m.group(1) if m else '?'}"
    if name.startswith("void "):
        name = name[5:]
    name = name.replace("(anonymous namespace)::", "")
    # drop the trailing argument list only (templates may contain parentheses)
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            name = name[:i]
            break
    return name[:120].replace("|", "/")


def _is_opt(name: str) -> bool:
    """One fused optimizer dispatch per training step: AdamW (GPT-2) or the
    momentum-SGD pass (ResNet-50)."""
    return "adamw" in name or "sgd_kernel" in name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=0,
                    help="traced steps (0: count the optimizer dispatches: fused AdamW or fused SGD)")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    t0 = min(r[2] for r in rows)
    t1 = max(r[3] for r in rows)
    for name, dur, _, _ in rows:
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += dur
    total = sum(v[1] for v in agg.values())
    if a.steps <= 0:
        # traced steps = optimizer dispatches (one fused AdamW per step); a plain
        # trace without an optimizer has no step column
        a.steps = sum(1 for r in rows if _is_opt(r[0]))
    print(f"# rocprofv3 kernel summary {a.title}\n")
    if a.steps:
        print(f"ms/step = total ms / {a.steps} traced steps (optimizer dispatches)\n")
    print(f"dispatches: {len(rows)}  kernel time: {total/1e6:.2f} ms  span: {(t1-t0)/1e6:.2f} ms\n")
    hdr = "| kernel | calls | total ms | mean us | % |"
    if a.steps:
        hdr = hdr[:-1] + " ms/step |"
    print(hdr)
    print("|" + "---|" * (hdr.count("|") - 1))
    for k, (n, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        line = f"| {k} | {n} | {d/1e6:.3f} | {d/n/1e3:.1f} | {100*d/total:.1f} |"
        if a.steps:
            line += f" {d/1e6/a.steps:.3f} |"
        print(line)
    # device idle inside the steady-state steps: steps end at the optimizer kernel
    # (one adamw dispatch per step); between the 2nd and the last one, busy = the
    # union of kernel intervals, idle = span - busy (launch gaps, host stalls)
    ends = sorted(r[3] for r in rows if _is_opt(r[0]))
    if len(ends) >= 4:
        lo, hi = ends[1], ends[-1]
        iv = sorted((max(s, lo), min(e, hi)) for _, _, s, e in rows if e > lo and s < hi)
        busy, cur_s, cur_e = 0, None, None
        for s, e in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        n = len(ends) - 2
        nk = sum(1 for _, _, s, e in rows if s >= lo and e <= hi)
        print(f"\nsteady state ({n} steps between optimizer kernels): {(hi - lo) / 1e6 / n:.3f} ms/step span, "
              f"{busy / 1e6 / n:.3f} busy, {(hi - lo - busy) / 1e6 / n:.3f} idle "
              f"({nk // n} dispatches/step, {(hi - lo - busy) / 1e3 / max(nk, 1):.2f} us idle per dispatch)")
    try:
        regs = c.execute("select name, start, end, extdata from regions").fetchall()
    except sqlite3.Error:
        regs = []
    if regs:
        # roctx ranges (utils/trace.py, PDO_ROCTX=1): host-side span of each phase
        # and the GPU kernel time that ran inside it (kernels are async, so the
        # GPU column shows how far the device lags the host)
        import json
        ph = defaultdict(lambda: [[], []])
        for name, s0, s1, ext in regs:
            try:
                msg = json.loads(ext).get("message", name)
            except (ValueError, TypeError):
                msg = name
            if msg.startswith("step "):
                msg = "step"
            busy = sum(min(e, s1) - max(s, s0) for _, _, s, e in rows if e > s0 and s < s1)
            ph[msg][0].append(s1 - s0)
            ph[msg][1].append(busy)
        print("\n## roctx phases (host span vs GPU kernel-busy time inside it)\n")
        med = lambda v: sorted(v)[len(v) // 2] / 1e6  # noqa: E731 (warm-up steps skew the mean)
        print("| phase | count | host ms (median) | GPU busy ms (median) |")
        print("|---|---|---|---|")
        for k, (d, b) in sorted(ph.items(), key=lambda x: -med(x[1][0])):
            print(f"| {k} | {len(d)} | {med(d):.2f} | {med(b):.2f} |")


if __name__ == "__main__":
    main()
