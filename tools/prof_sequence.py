#!/usr/bin/env python3
"""Kernel sequence of the last N dispatches of a rocprofv3 ``--kernel-trace``
database: name, duration and the idle gap before each kernel on the device.

usage: python tools/prof_sequence.py RUN_results.db [--last 700] [--gap-us 5]

Prints the total device-idle time inside the window (sum of gaps between
consecutive kernels) and the kernels that follow gaps above ``--gap-us`` —
the launch-bound spots of a step — plus the ordered list (markdown).
"""
import argparse
import sqlite3

from prof_summary import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=700)
    ap.add_argument("--gap-us", type=float, default=5.0)
    ap.add_argument("--list", action="store_true", help="print every kernel of the window")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()[-a.last:]
    busy = sum(e - s for _, s, e in rows)
    span = rows[-1][2] - rows[0][1]
    gaps = []
    prev_end = rows[0][1]
    for name, s, e in rows:
        gaps.append(max(0, s - prev_end))
        prev_end = max(prev_end, e)
    print(f"window: {len(rows)} kernels, span {span/1e6:.3f} ms, busy {busy/1e6:.3f} ms, "
          f"idle {sum(gaps)/1e6:.3f} ms\n")
    big = [(g, i) for i, g in enumerate(gaps) if g > a.gap_us * 1e3]
    print(f"gaps > {a.gap_us} us: {len(big)}, total {sum(g for g, _ in big)/1e6:.3f} ms\n")
    print("| gap us | before kernel | after kernel |\n|---|---|---|")
    for g, i in sorted(big, reverse=True)[:40]:
        print(f"| {g/1e3:.1f} | {short(rows[i][0])} | {short(rows[i-1][0]) if i else '-'} |")
    if a.list:
        print("\n| # | kernel | us | gap us |\n|---|---|---|---|")
        for i, (name, s, e) in enumerate(rows):
            print(f"| {i} | {short(name)} | {(e-s)/1e3:.1f} | {gaps[i]/1e3:.1f} |")


if __name__ == "__main__":
    main()
