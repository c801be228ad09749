#!/usr/bin/env python3
"""Build every native component of paddle_operator_amd in-tree.

* ``paddle_operator_amd/_pdo_hip.so`` — HIP kernels (csrc/hip/*.hip) compiled
  by ``hipcc --offload-arch=gfx950`` one object per file (no torch headers,
  seconds each) + ``bind.cpp`` (torch/pybind11 adapter), linked against the
  libtorch that will import it.  No hipify step, no CUDA names.
* ``paddle_operator_amd/_pdo_core.so`` and the ``bin/pdo-*`` executables —
  the native control plane (csrc/core, csrc/kv, csrc/manager, csrc/agent)
  built by CMake/Ninja.

Incremental: an object is rebuilt only when its source or any header in its
directory is newer.  ``--clean`` forces a full rebuild.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "paddle_operator_amd")
BUILD = os.path.join(ROOT, "build")
ARCH = os.environ.get("PDO_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _run(cmd, cwd=None):
    r = subprocess.run(cmd, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout)
        raise SystemExit(f"build step failed: {cmd[0]} (rc={r.returncode})")
    return r.stdout


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def torch_flags():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    import pybind11
    inc.append(pybind11.get_include())
    inc.append(sysconfig.get_paths()["include"])
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc] + [
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_pdo_hip", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
    ]
    lib = os.path.join(tdir, "lib")
    ldflags = [f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-ltorch_python", f"-Wl,-rpath,{lib}"]
    return cflags, ldflags


def build_hip(jobs=8, verbose=False):
    src_dir = os.path.join(ROOT, "csrc", "hip")
    obj_dir = os.path.join(BUILD, "hip")
    os.makedirs(obj_dir, exist_ok=True)
    headers = glob.glob(os.path.join(src_dir, "*.h"))
    kernels = sorted(glob.glob(os.path.join(src_dir, "*.hip")))
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
              "-Wno-unused-result", "-munsafe-fp-atomics"]
    # MFMA accumulators in arch VGPRs: no v_accvgpr copies around the VALU work
    # on accumulators (softmax / rescale / epilogues) — except where the
    # accumulators alone exceed the 256 arch VGPRs (gemm_nt4: 256 fp32 per lane
    # live in the accumulator file; the vgpr form made hipcc shuttle them
    # through arch VGPRs, 3 VALU per MFMA)
    vgpr_form = ["-mllvm", "-amdgpu-mfma-vgpr-form"]
    agpr_files = {"gemm_nt4.hip", "gemm_dw4.hip"}
    # per-file extras: attention's softmax max-reductions become v_max3 only
    # without NaN canonicalisation (scores are never NaN; ±inf masks keep working)
    extra = {"attention.hip": ["-fno-honor-nans"]}
    jobs_list = []
    for s in kernels:
        o = os.path.join(obj_dir, os.path.basename(s) + ".o")
        if _newer(o, [s] + headers + [os.path.abspath(__file__)]):
            form = [] if os.path.basename(s) in agpr_files else vgpr_form
            jobs_list.append([HIPCC] + common + form + extra.get(os.path.basename(s), []) + ["-c", s, "-o", o])
    tcf, tld = torch_flags()
    bind = os.path.join(src_dir, "bind.cpp")
    bind_o = os.path.join(obj_dir, "bind.o")
    if _newer(bind_o, [bind] + headers):
        jobs_list.append([HIPCC] + common + vgpr_form + tcf + ["-x", "hip", "-c", bind, "-o", bind_o])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    objs = [os.path.join(obj_dir, os.path.basename(s) + ".o") for s in kernels] + [bind_o]
    so = os.path.join(PKG, "_pdo_hip.so")
    if _newer(so, objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", so] + objs + tld)
    build_rccl_tools()
    return so


def build_rccl_tools():
    """bin/pdo-allreduce-bench: standalone RCCL bandwidth sweep (no torch)."""
    src = os.path.join(ROOT, "csrc", "rccl", "allreduce_bench.hip")
    exe = os.path.join(ROOT, "bin", "pdo-allreduce-bench")
    if not os.path.exists(src) or not _newer(exe, [src]):
        return exe
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    _run([HIPCC, "-O2", "-std=c++17", f"--offload-arch={ARCH}", src, "-o", exe, "-L/opt/rocm/lib", "-lrccl",
          "-Wl,-rpath,/opt/rocm/lib"])
    return exe


def build_core(jobs=8):
    """CMake build of the C++ control plane (+ pybind module)."""
    src = os.path.join(ROOT, "csrc")
    if not os.path.exists(os.path.join(src, "CMakeLists.txt")):
        return None
    bdir = os.path.join(BUILD, "core")
    os.makedirs(bdir, exist_ok=True)
    import pybind11
    if not os.path.exists(os.path.join(bdir, "build.ninja")):
        _run(["cmake", "-G", "Ninja", "-S", src, "-B", bdir, "-DCMAKE_BUILD_TYPE=Release",
              f"-Dpybind11_DIR={pybind11.get_cmake_dir()}",
              f"-DPython_EXECUTABLE={sys.executable}", f"-DPDO_PKG_DIR={PKG}",
              f"-DPDO_BIN_DIR={os.path.join(ROOT, 'bin')}"])
    _run(["cmake", "--build", bdir, "--", f"-j{jobs}"])
    return bdir


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--only", choices=["hip", "core"], default=None)
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    if a.clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    if a.only in (None, "core"):
        b = build_core(a.jobs)
        print(f"[build] core: {b}")
    if a.only in (None, "hip"):
        so = build_hip(a.jobs, a.verbose)
        print(f"[build] hip: {so}")


if __name__ == "__main__":
    main()
