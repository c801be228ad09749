#!/usr/bin/env python3
"""In-process GPT-2 training loop for profiling (rocprofv3 wraps THIS process).

bench.py launches its ranks through the operator (agent fork/exec), which a
profiler attached to bench.py would not follow; this probe runs the same
``GPT2Trainer`` step in one process so ``rocprofv3 -- python3
tools/train_probe.py`` sees every kernel.

    python tools/train_probe.py --model gpt2-medium --batch 64 --steps 5 --warmup 2
    PDO_DDP_ALWAYS=1 python tools/train_probe.py --dist ...   # RCCL bucket all-reduces at world 1
    torchrun --nproc-per-node 2 tools/train_probe.py --dist   # (PDO_DIST_BACKEND=gloo: 2 ranks, 1 GPU)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dist", action="store_true", help="init the (RCCL) process group even at world 1")
    ap.add_argument("--bucket-mb", type=int, default=0)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from paddle_operator_amd.models.gpt2 import GPT2Config
    from paddle_operator_amd.train import GPT2Trainer, init_distributed
    from paddle_operator_amd.utils import trace

    if a.dist:
        info = init_distributed()
        dev = torch.device("cuda", info.local_rank)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    cfg = GPT2Config.named(a.model)
    tr = GPT2Trainer(cfg, a.batch, a.seq, dev, bucket_mb=a.bucket_mb or None)
    tr.sync_initial_weights()
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        with trace.range(f"step {i}"):
            loss = tr.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    world = dist.get_world_size() if dist.is_initialized() else 1
    print(json.dumps({"model": a.model, "batch": a.batch, "ms_per_step": round(dt * 1e3, 3),
                      "tokens_per_s": round(a.batch * a.seq * world / dt, 1), "world": world,
                      "ddp_enabled": tr.ddp.enabled, "buckets": len(tr.flat.buckets),
                      "grad_reduce": tr.ddp.grad_reduce, "loss": float(loss)}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
