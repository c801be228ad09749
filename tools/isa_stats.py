#!/usr/bin/env python3
"""Instruction mix of HIP kernels, per basic block, from hipcc's gfx950 assembly.

Static counts only (a block's count × its trip count is what the hardware
issues); used next to rocprofv3 --pmc SQ_INSTS_* to see where VALU issue goes.

    python tools/isa_stats.py csrc/hip/attention.hip attn_fwd3 [--blocks]

Compiles the file with the flags tools/build.py uses (device only, -S) and
prints, per kernel whose mangled name contains the pattern: VGPR count and
totals by class (mfma / valu / exp / salu / ds / global / nop / waitcnt),
and with --blocks the same per basic block, marking loop blocks.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt")):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op == "s_nop":
        return "nop"
    if op == "s_waitcnt":
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return op.split("_")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("pattern")
    ap.add_argument("--blocks", action="store_true")
    ap.add_argument("--flags", default="")
    a = ap.parse_args()
    from tools.build import ARCH
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-munsafe-fp-atomics",
             "-mllvm", "-amdgpu-mfma-vgpr-form", "-I", os.path.join(ROOT, "csrc", "hip")]
    if os.path.basename(a.src) == "attention.hip":
        flags.append("-fno-honor-nans")
    flags += a.flags.split()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["--cuda-device-only", "-S", "-o", out, a.src], check=True,
                       stderr=subprocess.DEVNULL)
        s = open(out).read()
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        if a.pattern not in name:
            continue
        body = s[m.start():s.find(".Lfunc_end", m.start())]
        k = s.find(".amdhsa_kernel " + name)
        nv = re.search(r"amdhsa_next_free_vgpr (\d+)", s[k:]).group(1) if k >= 0 else "?"
        tot = collections.Counter()
        blocks, cur, label = [], collections.Counter(), "entry"
        for line in body.split("\n"):
            t = line.strip()
            if t.startswith(".LBB") or t.startswith("; %bb."):
                blocks.append((label, cur))
                label, cur = t, collections.Counter()
                continue
            if not t or t[0] in ";.":
                continue
            c = classify(t.split()[0])
            cur[c] += 1
            tot[c] += 1
        blocks.append((label, cur))
        print(f"{name}  vgpr={nv}  " + " ".join(f"{k}={v}" for k, v in sorted(tot.items())))
        if a.blocks:
            for lab, c in blocks:
                if c:
                    print(f"   {lab[:60]:60s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
