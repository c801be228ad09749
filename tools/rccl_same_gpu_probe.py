#!/usr/bin/env python3
"""Can two RCCL ranks share one GPU on this image?  (2 processes, 1 device)

Prints one JSON line {"ok": bool, "error": ...}.  Each rank all-reduces a
tensor; a hang is bounded by the process-group timeout (30 s)."""
import datetime
import json
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port, q):
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2,
                                timeout=datetime.timedelta(seconds=30), device_id=torch.device("cuda", 0))
        t = torch.full((1 << 20,), float(rank + 1), device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        q.put((rank, float(t[0]), None))
        dist.destroy_process_group()
    except Exception as e:  # report, do not hang
        q.put((rank, None, repr(e)[:500]))


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = []
    for _ in range(2):
        try:
            res.append(q.get(timeout=90))
        except Exception as e:
            res.append((None, None, f"timeout: {e!r}"))
    for p in ps:
        p.join(30)
        if p.is_alive():
            p.kill()
    ok = all(r[1] == 3.0 for r in res)
    print(json.dumps({"ok": ok, "results": res}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
