#!/usr/bin/env python3
"""Does a cached RCCL topology (NCCL_TOPO_FILE, dumped by an earlier communicator
of the same process via NCCL_TOPO_DUMP_FILE) shorten a warm rank's communicator
init?  Prints the timed inits; run with NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT to
get RCCL's own 'Init timings' lines.

    python tools/rccl_topo_probe.py [--channels N]
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def once(dev, x):
    t0 = time.time()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=dev)
    t1 = time.time()
    dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.destroy_process_group()
    return round(t1 - t0, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "pdo_rccl_topo.xml"))
    a = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    x = torch.ones(1, device=dev)
    os.environ["NCCL_TOPO_DUMP_FILE"] = a.out
    first = once(dev, x)
    del os.environ["NCCL_TOPO_DUMP_FILE"]
    res = {"first": first, "dump_exists": os.path.exists(a.out)}
    res["warm_default"] = [once(dev, x) for _ in range(3)]
    os.environ["NCCL_TOPO_FILE"] = a.out
    res["warm_topo_file"] = [once(dev, x) for _ in range(3)]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
