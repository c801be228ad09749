#!/usr/bin/env python3
"""RCCL ↔ compute overlap from a rocprofv3 ``--kernel-trace`` database.

usage: python tools/overlap_summary.py <run_results.db> [--title T]

Classifies each dispatch as communication (RCCL kernels: names containing
``nccl``/``rccl``) or compute, and reports per RCCL kernel how much of its
[start, end] interval is covered by compute kernels running concurrently
(on other queues), plus the totals.  Markdown output for ``profiles/``.
"""
import argparse
import sqlite3


def is_comm(name):
    n = name.lower()
    return "nccl" in n or "rccl" in n


def merge(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(s, e, merged):
    tot = 0
    for a, b in merged:
        if b <= s:
            continue
        if a >= e:
            break
        tot += min(b, e) - max(a, s)
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    comm = [(n, s, e) for n, s, e in rows if is_comm(n)]
    comp = merge([[s, e] for n, s, e in rows if not is_comm(n)])
    print(f"# RCCL / compute overlap {a.title}\n")
    print(f"dispatches: {len(rows)}, RCCL kernels: {len(comm)}\n")
    if not comm:
        print("No RCCL kernels in the trace.")
        return
    names = {}
    tot_d = tot_o = 0
    for n, s, e in comm:
        d = e - s
        o = covered(s, e, comp)
        k = n.split("(")[0][:90]
        x = names.setdefault(k, [0, 0, 0])
        x[0] += 1
        x[1] += d
        x[2] += o
        tot_d += d
        tot_o += o
    print("| RCCL kernel | calls | total us | overlapped with compute us | % overlapped |")
    print("|---|---|---|---|---|")
    for k, (cnt, d, o) in sorted(names.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {cnt} | {d/1e3:.1f} | {o/1e3:.1f} | {100*o/max(d,1):.1f} |")
    print(f"\n**total RCCL kernel time {tot_d/1e6:.3f} ms, {100*tot_o/max(tot_d,1):.1f}% of it concurrent with "
          f"compute kernels**\n")
    print("First 12 RCCL dispatches (µs from trace start) with the compute kernel running at their start:\n")
    t0 = rows[0][1]
    print("| # | RCCL kernel | start us | dur us | concurrent compute kernel |")
    print("|---|---|---|---|---|")
    for i, (n, s, e) in enumerate(comm[:12]):
        conc = [cn for cn, cs, ce in rows if not is_comm(cn) and cs <= s < ce]
        print(f"| {i} | `{n.split('(')[0][:50]}` | {(s-t0)/1e3:.1f} | {(e-s)/1e3:.1f} | "
              f"`{(conc[0].split('(')[0][:60]) if conc else '-'}` |")


if __name__ == "__main__":
    main()
