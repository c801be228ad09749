"""Checkpoint / resume for launched jobs (SURVEY §5.4 [design]).

The reference leaves this to the user script (deploy/elastic/resnet.yaml
mounts hostPath /checkpoint).  pdo-launch saves model + optimizer + step from
rank 0 every ``--ckpt-every`` steps and on SIGTERM, atomically (write to a
temp file, fsync, rename), keeps the last ``keep`` checkpoints, and resumes
from the newest one on (re)start — including after an elastic re-rendezvous
at a different world size (the flat arena layout does not depend on world).
"""
from __future__ import annotations

import glob
import os
import re
from typing import Optional, Tuple

import torch

_PAT = re.compile(r"ckpt-(\d+)\.pt$")


def save(state: dict, ckpt_dir: str, step: int, keep: int = 2) -> str:
    os.makedirs(ckpt_dir, exist_ok=True)
    path = os.path.join(ckpt_dir, f"ckpt-{step:08d}.pt")
    tmp = path + f".tmp{os.getpid()}"
    cpu_state = {k: (v.detach().cpu() if torch.is_tensor(v) else v) for k, v in state.items()}
    cpu_state["step"] = step
    with open(tmp, "wb") as f:
        torch.save(cpu_state, f)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    for old in sorted(glob.glob(os.path.join(ckpt_dir, "ckpt-*.pt")))[:-keep]:
        try:
            os.remove(old)
        except OSError:
            pass
    return path


def latest(ckpt_dir: str) -> Optional[str]:
    if not ckpt_dir or not os.path.isdir(ckpt_dir):
        return None
    c = [p for p in glob.glob(os.path.join(ckpt_dir, "ckpt-*.pt")) if _PAT.search(p)]
    return max(c, key=lambda p: int(_PAT.search(p).group(1))) if c else None


def load_latest(ckpt_dir: str, map_location="cpu") -> Tuple[Optional[dict], int]:
    p = latest(ckpt_dir)
    if p is None:
        return None, 0
    st = torch.load(p, map_location=map_location, weights_only=True)
    return st, int(st.get("step", 0))
