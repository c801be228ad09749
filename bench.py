#!/usr/bin/env python3
"""Headline benchmark: launched GPT-2-medium training throughput on MI355X.

BASELINE.json metric: "job-start->all-ranks-ready p50 (s); launched tokens/sec
at 1/2/4/8 MI355X".  This script measures the flagship *training step* of a
launched collective-mode job (config 4: GPT-2-medium, seq 1024, bf16, data
parallel over RCCL/xGMI, one rank per GPU) and reports the whole-job
tokens/s.  The time from process start until every rank is ready (RCCL
communicator up, weights broadcast, first barrier passed) is reported as
``ready_s`` alongside.  The operator-level launch latency (PaddleJob →
all-ranks-ready through the control plane) is measured by
``python bench_launch.py``.

Per-GPU micro-batch 64 × 1024 tokens (weak scaling): at 8 GPUs the global
batch is 512 sequences = 0.5 M tokens, GPT-2's own batch size; GEMM shapes
are pre-tuned for it (paddle_operator_amd/tuning/*_b64_gfx950.csv).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
it runs under ``torch.distributed.run`` one rank per GPU.  W untimed steps,
then exactly K timed steps bracketed by barrier + device synchronize; the max
over ranks is reported by rank 0 as one JSON line.

Data: synthetic tokens generated on device each step; weights: random init.
"""
import time

_T0 = time.time()  # process start (before torch import) for ready_s

import argparse  # noqa: E402
import json  # noqa: E402
import os  # noqa: E402
import sys  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--micro-batch", type=int, default=int(os.environ.get("PDO_MICRO_BATCH", "64")))
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--bucket-mb", type=int, default=64)
    ap.add_argument("--ops", choices=["hip", "torch"], default=os.environ.get("PDO_OPS", "hip"))
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args()
    os.environ["PDO_OPS"] = args.ops

    import torch
    import torch.distributed as dist
    from paddle_operator_amd.models.gpt2 import GPT2Config
    from paddle_operator_amd.train import GPT2Trainer, init_distributed

    info = init_distributed()
    world = info.world
    if world != args.gpus and info.is_main:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    dev = torch.device("cuda", info.local_rank) if torch.cuda.is_available() else torch.device("cpu")
    cfg = GPT2Config.named(args.model)
    tr = GPT2Trainer(cfg, args.micro_batch, args.seq, dev, bucket_mb=args.bucket_mb)
    tr.sync_initial_weights()

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def barrier():
        if dist.is_initialized():
            dist.barrier()

    sync()
    barrier()
    t_ready = time.time()

    for _ in range(args.warmup):
        loss = tr.step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = tr.step()
    sync()
    barrier()
    sync()
    dt = time.perf_counter() - t0
    loss_v = float(loss.detach().float().item())

    # max over ranks of elapsed time; ready = latest ready minus earliest start
    vals = torch.tensor([dt, t_ready, -_T0], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
    dt = float(vals[0])
    ready_s = float(vals[1]) + float(vals[2])

    tokens = tr.tokens_per_step() * world * args.steps
    tps = tokens / dt
    ms = dt / args.steps * 1e3
    flops = cfg.flops_per_token(args.seq) * tps / world
    if info.is_main:
        rec = {
            "metric": "launched tokens/sec (GPT-2-medium collective DP, bf16)",
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (on-device random tokens), random-init weights",
            "config": {
                "model": args.model,
                "global_batch": args.micro_batch * world,
                "micro_batch_per_gpu": args.micro_batch,
                "seq_len": args.seq,
                "parallelism": f"dp{world}",
                "bucket_mb": args.bucket_mb,
                "ops": args.ops,
            },
            "ready_s": round(ready_s, 3),
            "model_tflops_per_gpu": round(flops / 1e12, 1),
            "mfu_vs_2.5PF_dense": round(flops / 2.5e15, 4),
            "final_loss": round(loss_v, 4),
        }
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
