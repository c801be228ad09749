"""Pre-tuned hipBLASLt/rocBLAS GEMM selection (PyTorch TunableOp) for gfx950.

The flagship steps' GEMMs run on the hand-written gemm_nt4 / gemm_dw4 kernels;
library GEMMs remain for shapes outside their contracts, the tiny classifier
heads and the framework reference path (PDO_OPS=torch).  For those, instead of
hipBLASLt's heuristic pick, every GEMM shape of the flagship step was benchmarked once on
an MI355X (all hipBLASLt + rocBLAS solutions, TunableOp) and the winners are
shipped in ``paddle_operator_amd/tuning/*.csv`` (validated against the
PyTorch/HIP/hipBLASLt versions and the gcnArchName recorded in the file).
At start-up every rank loads the table with tuning disabled: no benchmarking
inside a training job, identical kernel choice on every rank.

``PDO_TUNE_GEMMS=1`` switches online tuning on (new shapes are benchmarked at
first use and appended to ``PDO_TUNE_OUT``).
"""
from __future__ import annotations

import glob
import os
import shutil

import torch

_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def tuned_tables():
    return sorted(glob.glob(os.path.join(_DIR, "tunableop_*_gfx950.csv")))


def enable_tuned_gemms(verbose: bool = False) -> int:
    """Load every shipped table; returns the number of tables read."""
    if not torch.cuda.is_available():
        return 0
    tun = torch.cuda.tunable
    tun.enable(True)
    online = os.environ.get("PDO_TUNE_GEMMS", "0") == "1"
    tun.tuning_enable(online)
    if online:
        tun.set_filename(os.environ.get("PDO_TUNE_OUT", "/tmp/pdo_tunableop%d.csv"))
        tun.set_max_tuning_duration(int(os.environ.get("PDO_TUNE_MS", "100")))
    n = 0
    for f in tuned_tables():
        try:
            if tun.read_file(f):
                n += 1
        except Exception as e:  # validator mismatch (different ROCm / torch build)
            if verbose:
                print(f"[pdo] tuning table {os.path.basename(f)} not loaded: {e}")
    if verbose:
        print(f"[pdo] tuned GEMM tables loaded: {n}")
    return n


def use_shipped_miopen_db(verbose: bool = False) -> str | None:
    """Point MIOpen's user find-db/perf-db at a private copy of the shipped
    gfx950 convolution find results (``tuning/miopen/*``), before the first
    convolution creates a MIOpen handle.  A user-set ``MIOPEN_USER_DB_PATH`` is
    left alone.  Returns the db directory in use (None if nothing shipped)."""
    if os.environ.get("MIOPEN_USER_DB_PATH"):
        return os.environ["MIOPEN_USER_DB_PATH"]
    src = os.path.join(_DIR, "miopen")
    files = [f for f in glob.glob(os.path.join(src, "*")) if os.path.isfile(f)]
    if not files:
        return None
    dst = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"pdo-miopen-{os.getuid()}")
    os.makedirs(dst, exist_ok=True)
    for f in files:
        t = os.path.join(dst, os.path.basename(f))
        if not os.path.exists(t) or os.path.getmtime(t) < os.path.getmtime(f):
            tmp = f"{t}.{os.getpid()}"
            shutil.copy2(f, tmp)  # MIOpen appends to its user db: never hand it the tracked file
            os.replace(tmp, t)  # atomic: ranks of one node share the directory
    os.environ["MIOPEN_USER_DB_PATH"] = dst
    if verbose:
        print(f"[pdo] MIOpen user db: {dst} ({len(files)} shipped files)")
    return dst
