#!/usr/bin/env python3
"""Per-(kernel, grid) breakdown of a rocprofv3 kernel-trace database: separates
the GEMM shapes that share one library kernel (grid size tells them apart).

    python tools/prof_shapes.py gpurun_out/<run>/prof/run_results.db [--match Cijk] [--steps 7]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--steps", type=int, default=7, help="steps in the trace (calls per step = calls / steps)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = collections.defaultdict(list)
    for name, gx, gy, gz, dur in c.execute("select name, grid_x, grid_y, grid_z, duration from kernels"):
        if a.match and a.match not in name:
            continue
        agg[(name[:70], gx, gy, gz)].append(dur / 1e3)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    print("| kernel | grid | calls/step | mean µs | ms/step |")
    print("|---|---|---|---|---|")
    for (name, gx, gy, gz), d in rows[:40]:
        print(f"| {name} | {gx}x{gy}x{gz} | {len(d) / a.steps:.1f} | {sum(d) / len(d):.1f} | {sum(d) / a.steps / 1e3:.3f} |")


if __name__ == "__main__":
    main()
