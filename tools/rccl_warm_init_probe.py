#!/usr/bin/env python3
"""A warm process's SECOND 1-rank RCCL communicator (what a GPU-warm slot's rank
pays): build + destroy one communicator, then time init_process_group + first
all-reduce again, with RCCL's INIT log timestamped by this process (stderr is
re-read through a pipe).  Env knobs under test pass through (NCCL_TOPO_FILE …).

    NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT python tools/rccl_warm_init_probe.py
"""
import json
import os
import threading
import time

r, w = os.pipe()
saved = os.dup(2)
os.dup2(w, 2)
lines = []


def _reader():
    with os.fdopen(r, "r", errors="replace") as f:
        for line in f:
            lines.append((time.time(), line.rstrip()))


th = threading.Thread(target=_reader, daemon=True)
th.start()

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.cuda.set_device(0)
torch.cuda.init()
dev = torch.device("cuda", 0)
x = torch.ones(1, device=dev)


def once():
    t0 = time.time()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    t1 = time.time()
    dist.all_reduce(x)
    torch.cuda.synchronize()
    t2 = time.time()
    dist.destroy_process_group()
    return t0, t1, t2


once()
mark = time.time()
t0, t1, t2 = once()
time.sleep(0.2)
os.dup2(saved, 2)
res = {"warm_pg_init_s": round(t1 - t0, 4), "warm_first_allreduce_s": round(t2 - t1, 4)}
print(json.dumps(res), flush=True)
for t, l in lines:
    if t >= mark:
        print(f"{(t - t0) * 1e3:8.2f} ms  {l[:160]}")
