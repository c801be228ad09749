"""Bucketed, backward-overlapped gradient all-reduce over RCCL (xGMI).

Collective-mode data parallelism for PaddleJobs (``Mode=Collective``,
reference ``controllers/paddlejob_helper.go:191-199``; the reference leaves the
NCCL all-reduce to the Paddle image).  Design for MI355X:

* gradients live in the flat arena (``parallel.flat``): a bucket is a slice,
  so the all-reduce runs on the gradient memory itself (no flatten copy);
* a post-accumulate-grad hook counts ready parameters per bucket and launches
  ``all_reduce(SUM)`` on the bucket as soon as it is complete — RCCL runs on
  its own HIP stream, overlapping the backward GEMMs of the earlier layers;
* the 1/world average is NOT a separate scale kernel: it is folded into the
  fused AdamW step (``grad_scale``);
* bucket size defaults to 64 MiB: on 8×MI355X each ring step moves
  bucket/8 per link and 7 xGMI links run concurrent channels, so buckets below
  ~16 MiB fall off the bandwidth plateau while buckets above ~128 MiB delay the
  first overlap (see ``tools/allreduce_sweep.py`` / ``profiles/``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .flat import FlatParams


class BucketedDDP:
    def __init__(self, flat: FlatParams, group=None, enabled: bool | None = None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.enabled = (self.world > 1) if enabled is None else enabled
        self._pending = [0] * len(flat.buckets)
        self._sizes = [len(b.slots) for b in flat.buckets]
        self._works = []
        self._sync = True
        self._launched = [False] * len(flat.buckets)
        self._next = 0
        self._bucket_of = flat.bucket_of()
        self._seen = set()
        self._hooks = []
        if self.enabled:
            for s in flat.slots:
                self._hooks.append(s.param.register_post_accumulate_grad_hook(self._hook))
                # ops that write gradients straight into the arena signal here
                s.param._pdo_ready = self._hook

    # -- API --------------------------------------------------------------
    def broadcast_params(self, src: int = 0):
        """Make every rank start from rank ``src``'s weights (one collective)."""
        if self.world > 1:
            dist.broadcast(self.flat.params, src, group=self.group)

    def no_sync(self):
        ddp = self

        class _Ctx:
            def __enter__(self):
                ddp._sync = False

            def __exit__(self, *a):
                ddp._sync = True
        return _Ctx()

    def prepare(self):
        """Call before backward: reset per-step bucket bookkeeping."""
        self._pending = [0] * len(self.flat.buckets)
        self._launched = [False] * len(self.flat.buckets)
        self._works = []
        self._next = 0
        self._seen = set()

    def finish(self):
        """Call after backward: launch stragglers, make the compute stream wait."""
        if not (self.enabled and self._sync):
            return
        while self._next < len(self.flat.buckets):
            self._launch(self._next)
        for w in self._works:
            w.wait()
        self._works = []

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world if self.enabled else 1.0

    # -- internals ----------------------------------------------------------
    def _hook(self, p):
        """Readiness of one parameter's gradient for this step.

        Two sources call it: the post-accumulate-grad hook and, for gradients
        a kernel wrote straight into the arena, the op itself (``p._pdo_ready``)
        right after enqueuing that kernel.  The autograd engine ALSO runs the
        post-accumulate hook for such a parameter although its Function
        returned no gradient, so each parameter counts once per step — a
        double count would launch its bucket's all-reduce before the rest of
        the bucket was written (caught by tests/test_ddp_gpu.py)."""
        if not self._sync:
            return
        key = id(p)
        if key in self._seen:
            return
        self._seen.add(key)
        i = self._bucket_of[key]
        self._pending[i] += 1
        # buckets are issued strictly in index order (identical on every rank,
        # whatever order the autograd engine produced the gradients in)
        n = len(self._sizes)
        while self._next < n and self._pending[self._next] == self._sizes[self._next]:
            self._launch(self._next)

    def _launch(self, i):
        b = self.flat.buckets[i]
        self._launched[i] = True
        self._next = i + 1
        w = dist.all_reduce(self.flat.grads[b.start:b.end], op=dist.ReduceOp.SUM,
                            group=self.group, async_op=True)
        self._works.append(w)
