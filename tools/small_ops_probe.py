#!/usr/bin/env python3
"""Where the GPT-2 step's small framework kernels come from.

Runs the GPT-2-medium training step in one process, then profiles one step
with ``torch.profiler`` and prints every aten op that launched a fill / copy /
memset / elementwise kernel, with the innermost paddle_operator_amd frame of
its Python stack — the source line to fuse or delete.

    python tools/small_ops_probe.py [--model gpt2-medium] [--batch 64]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=1024)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from paddle_operator_amd.models.gpt2 import GPT2Config
    from paddle_operator_amd.train import GPT2Trainer, init_distributed

    info = init_distributed()
    dev = torch.device("cuda", info.local_rank)
    tr = GPT2Trainer(GPT2Config.named(a.model), a.batch, a.seq, dev)
    tr.sync_initial_weights()
    for _ in range(2):
        tr.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step()
        torch.cuda.synchronize()
    keep = ("fill", "copy", "zero", "memset", "Memcpy", "Memset", "add", "mul", "sum", "stack", "ones", "zeros",
            "to", "cat", "clamp", "div", "randint", "sort", "index", "empty_like")
    where = collections.Counter()
    for ev in prof.events():
        if ev.device_type.name != "CPU" or not ev.name.startswith("aten::"):
            continue
        if not any(k in ev.name for k in keep):
            continue
        if not ev.kernels and ev.device_time_total <= 0:
            continue
        frame = "?"
        for f in ev.stack or []:
            if "paddle_operator_amd" in f or "bench" in f or "tools/" in f:
                frame = f
                break
        where[(ev.name, frame)] += 1
    print("count | aten op | innermost repo frame")
    for (name, frame), n in where.most_common():
        print(f"{n:4d} | {name} | {frame}")
    ka = prof.key_averages()
    print(ka.table(sort_by="device_time_total", row_limit=40))


if __name__ == "__main__":
    main()
