"""Training step engine shared by ``bench.py``, ``pdo-launch`` workloads and tests.

One step = zero grads (memset of the flat arena) → forward → backward with
bucketed RCCL all-reduce overlapped → fused AdamW.  Synthetic batches are
generated on device every step (``torch.randint`` on the GPU; no H2D copy),
matching BASELINE's "synthetic data / random-init weights" rule.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from .models.gpt2 import GPT2, GPT2Config
from .ops import deferred_reductions
from .ops.optim import FlatAdamW
from .parallel.ddp import BucketedDDP
from .parallel.flat import FlatParams
from .utils import trace
from .utils.topology import bucket_bytes_for


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def is_main(self):
        return self.rank == 0


def init_distributed(backend: str | None = None, timeout_s: int = 600) -> DistInfo:
    """Initialise torch.distributed from the torchrun / pdo-launch env contract.

    On ROCm the ``nccl`` backend IS RCCL.  ``hipSetDevice(local_rank)`` happens
    before any other HIP call so the communicator binds the right GPU.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    info = DistInfo(rank, world, local)
    # PDO_DIST_BACKEND=gloo rehearses the multi-rank GPU path with every rank on
    # one device (RCCL refuses two ranks per GPU); production is nccl = RCCL
    backend = backend or os.environ.get("PDO_DIST_BACKEND") or None
    if torch.cuda.is_available():
        ndev = torch.cuda.device_count()
        if backend == "gloo" and local >= ndev:
            local = local % ndev
            info.local_rank = local
        torch.cuda.set_device(local)
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    # RCCL comes up eagerly even at world 1 (device_id → communicator built
    # now, so "ready" includes comm init and the DDP path is the one that runs
    # at scale); a CPU world of 1 needs no process group
    if (world > 1 or backend == "nccl") and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        if world == 1 and "MASTER_PORT" not in os.environ:
            kw["store"] = dist.HashStore()  # single rank: no rendezvous port
        import datetime
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return info


class GPT2Trainer:
    def __init__(self, cfg: GPT2Config, micro_batch: int, seq_len: int, device,
                 dtype=torch.bfloat16, lr=3e-4, bucket_mb: int | None = None, seed: int = 0):
        self.cfg = cfg
        self.B = micro_batch
        self.S = seq_len
        self.device = torch.device(device)
        if self.device.type == "cuda":
            from .utils.tuning import enable_tuned_gemms
            enable_tuned_gemms()
        torch.manual_seed(seed)
        if self.device.type == "cuda":
            # built and initialised on the device (models/gpt2.py reset_parameters)
            with torch.device(self.device):
                model = GPT2(cfg)
        else:
            model = GPT2(cfg)
        model.to(device=self.device, dtype=dtype)
        self.model = model
        if bucket_mb is None:
            world = dist.get_world_size() if dist.is_initialized() else 1
            nbytes = sum(p.numel() for p in model.parameters()) * torch.empty((), dtype=dtype).element_size()
            bucket_bytes = bucket_bytes_for(world, nbytes)
        else:
            bucket_bytes = bucket_mb << 20
        # the tied wte gradient in two slots: the LM-head half is bucket 0 (its
        # all-reduce overlaps the whole backward), the embedding half the last
        # bucket (PDO_SPLIT_WTE=0: one slot, all of it in the last bucket)
        split = ("wte",) if os.environ.get("PDO_SPLIT_WTE", "1") != "0" else ()
        self.flat = FlatParams(model, dtype=dtype, device=self.device, bucket_bytes=bucket_bytes, late=("wte",),
                               split=split)
        # every dX GEMM's Wᵀ operand built in one launch per step (wt_scope)
        self.flat.enable_wt()
        self.ddp = BucketedDDP(self.flat)
        self.opt = FlatAdamW(self.flat, lr=lr)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed + (dist.get_rank() if dist.is_initialized() else 0))

    def sync_initial_weights(self):
        self.ddp.broadcast_params(0)
        self.opt.master.copy_(self.flat.params.float())

    def batch(self):
        V = self.cfg.vocab_size
        idx = torch.randint(0, V, (self.B, self.S + 1), device=self.device, generator=self.gen)
        return idx[:, :-1], idx[:, 1:]

    def step(self, idx=None, tgt=None):
        if idx is None:
            idx, tgt = self.batch()
        self.flat.zero_grad()
        self.ddp.prepare()
        with self.flat.wt_scope():
            with trace.range("forward"):
                loss = self.model(idx, tgt)
            # bias / norm-weight column sums batched (flushed before each bucket
            # all-reduce and at the end of the backward)
            with trace.range("backward"), deferred_reductions(self.device):
                loss.backward()
        with trace.range("allreduce_drain"):
            self.ddp.finish(self.opt if self.opt.max_grad_norm else None)
        with trace.range("optimizer"):
            self.opt.step(grad_scale=self.ddp.grad_scale)
        return loss

    def tokens_per_step(self):
        return self.B * self.S


def now():
    return time.perf_counter()
