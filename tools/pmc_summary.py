#!/usr/bin/env python3
"""Per-kernel PMC counter averages from rocprofv3 rocpd databases.

usage: python tools/pmc_summary.py gpurun_out/pmc1/run_results.db [more.db ...] [--filter attn]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    table = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for db in a.dbs:
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        rows = c.execute("select * from counters_collection").fetchall()
        for r in rows:
            d = dict(zip(cols, r))
            name = d.get("kernel_name") or d.get("name") or ""
            if a.filter and a.filter not in name:
                continue
            table[name][d["counter_name"]].append(d["value"])
        kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        for r in c.execute("select * from kernels").fetchall():
            d = dict(zip(kcols, r))
            name = d.get("name") or d.get("kernel_name") or ""
            if a.filter and a.filter not in name:
                continue
            durs[name].append((d["end"] - d["start"]) / 1e3)
    for name, ctr in table.items():
        short = name.split("(")[0][:60]
        dd = durs.get(name, [])
        print(f"## {short}  (dispatches {len(dd)}, mean {sum(dd)/max(1,len(dd)):.1f} us)")
        for k in sorted(ctr):
            v = ctr[k]
            print(f"  {k:28s} {sum(v)/len(v):.4g}")


if __name__ == "__main__":
    main()
