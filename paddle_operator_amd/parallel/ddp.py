"""Bucketed, backward-overlapped gradient all-reduce over RCCL (xGMI).

Collective-mode data parallelism for PaddleJobs (``Mode=Collective``,
reference ``controllers/paddlejob_helper.go:191-199``; the reference leaves the
NCCL all-reduce to the Paddle image).  Design for MI355X:

* gradients live in the flat arena (``parallel.flat``): a bucket is a slice,
  so the all-reduce runs on the gradient memory itself (no flatten copy);
* a post-accumulate-grad hook counts ready parameters per bucket and launches
  ``all_reduce(SUM)`` on the bucket as soon as it is complete — RCCL runs on
  its own HIP stream, overlapping the backward GEMMs of the earlier layers;
* bucket size: ``utils.topology.bucket_bytes_for`` (a link-model heuristic,
  see its docstring; the callers pass it in);
* the tied embedding's gradient is split (``FlatParams(split=("wte",))``): the
  LM-head half is bucket 0, all-reduced as soon as the LM head's backward has
  written it, so it overlaps the whole backward instead of waiting for the
  embedding backward at the very end (the last bucket keeps only the
  embedding half);
* reduction precision (``grad_reduce``):

  - ``"bf16"`` (default for a bf16 arena): RCCL sums the bf16 bucket in
    place; the 1/world average is folded into the fused AdamW step
    (``grad_scale``).  Half the xGMI bytes of fp32.  The gradients are already
    bf16-rounded by the dW GEMM epilogue; the ring adds at most ``world − 1``
    more roundings of partial sums.  tests/test_ddp.py::
    test_grad_reduce_precision_4_ranks pins the effect at 4 ranks: the bf16-wire
    DDP gradient is within 1.5× of a single process's full-batch bf16 error
    against the fp32 reference.
  - ``"fp32"``: each bucket is cast to an fp32 staging arena with the 1/world
    average folded in (``cast_scale_bf16_f32``, csrc/hip/bucket.hip), reduced
    in fp32, and cast back into the bf16 arena once after the drain — one
    rounding of the exact average.  2× wire bytes + ~0.35 ms of HBM passes per
    GPT-2-medium step.  Select with ``PDO_GRAD_REDUCE=fp32``.

  An fp32 arena (ResNet-50) always reduces in fp32.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .flat import FlatParams


class BucketedDDP:
    def __init__(self, flat: FlatParams, group=None, enabled: bool | None = None, grad_reduce: str | None = None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        if enabled is None:
            # PDO_DDP_ALWAYS=1: reduce even at world 1 (RCCL overlap traces on one GPU)
            enabled = self.world > 1 or (os.environ.get("PDO_DDP_ALWAYS") == "1" and dist.is_initialized())
        self.enabled = enabled
        mode = grad_reduce or os.environ.get("PDO_GRAD_REDUCE") or "bf16"
        if mode not in ("bf16", "fp32"):
            raise ValueError(f"grad_reduce must be bf16 or fp32, not {mode!r}")
        # an fp32 arena is reduced in fp32 either way (no staging needed)
        self.stage = None
        if mode == "fp32" and flat.dtype != torch.float32 and self.enabled:
            self.stage = torch.zeros(flat.grads.numel(), dtype=torch.float32, device=flat.device)
        self.grad_reduce = "fp32" if (mode == "fp32" or flat.dtype == torch.float32) else "bf16"
        self._pending = [0] * len(flat.buckets)
        self._sizes = [len(b.slots) for b in flat.buckets]
        self._works = []
        self._work_bucket = []
        self._sync = True
        # first arena element the post-drain fold of a split gradient rewrites
        owners = {a.name[:-len("#head")] for a in flat.aux_slots}
        self._fold_start = min([s.offset for s in flat.slots if s.name in owners], default=flat.numel)
        self._launched = [False] * len(flat.buckets)
        self._next = 0
        self._bucket_of = flat.bucket_of()
        self._seen = set()
        self._hooks = []
        self._staged = False
        # gloo on GPU tensors (the shared-GPU rehearsal, PDO_DIST_BACKEND=gloo):
        # one bucket in flight at a time.  Dozens of queued async gloo all-reduces
        # on CUDA tensors collapsed to ~30 MB/s at 3 ranks (22 s per GPT-2-medium
        # step vs 2.4 GB/s for one-at-a-time all-reduces, bench.py
        # --rehearse-shared-gpu) and stalled outright at 4.  RCCL keeps the
        # overlapped pipeline: its collectives are stream-ordered kernels.
        self._serial = (self.enabled and flat.device.type == "cuda" and dist.is_initialized()
                        and dist.get_backend(group) == "gloo")
        if self.enabled:
            for s in flat.slots:
                self._hooks.append(s.param.register_post_accumulate_grad_hook(self._hook))
                # ops that write gradients straight into the arena signal here
                s.param._pdo_ready = self._hook
            for a in flat.aux_slots:  # a split parameter's head-gradient slot (bucket 0)
                a.param.ready = self._hook

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
        self._work_bucket = []
        self._next = 0
        self._seen = set()
        self._staged = False
        for a in self.flat.aux_slots:  # LM-head nodes writing a split slot this step (flat.AuxGrad)
            a.param.nodes = 0

    def finish(self, opt=None):
        """Call after backward: launch stragglers, make the compute stream wait,
        then fold split parameters' head-gradient slots into their gradients.

        ``opt`` (a FlatAdamW with clipping): its global-norm partials of each
        parameter bucket are queued right behind that bucket's wait, so they run
        while later buckets — the tied embedding's 105 MB tail last — are still
        on the wire; only the ranges the fold or the fp32 cast-back rewrite after
        the drain wait for the optimizer step."""
        _flush_reductions(buf_device=self.flat.device)
        if self.enabled and self._sync:
            while self._next < len(self.flat.buckets):
                self._launch(self._next)
            limit = 0 if self.stage is not None or opt is None else self._fold_start
            if opt is not None:
                opt.norm_reset()
            # collectives on one communicator complete in issue order; parameter
            # buckets are issued in ascending arena order
            for i, w in zip(self._work_bucket, self._works):
                w.wait()
                b = self.flat.buckets[i]
                if limit and b.start < self.flat.numel:
                    opt.norm_partial(min(b.end, limit))
            self._works = []
            self._work_bucket = []
            if self._staged:
                self._cast_back()
        self.flat.fold_split()

    @property
    def grad_scale(self) -> float:
        """Factor the optimizer applies to the arena gradients (1/world unless
        the average was already folded into the fp32 staging cast)."""
        if not self.enabled or self.stage is not None:
            return 1.0
        return 1.0 / self.world

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
        # queued bias / norm-weight column sums land in the arena first
        # (ops.deferred_reductions; stream-ordered before the all-reduce)
        _flush_reductions(buf_device=self.flat.device)
        self._launched[i] = True
        self._next = i + 1
        buf = self.flat.grads[b.start:b.end]
        if self.stage is not None:
            # fp32 wire: stage = grad / world on the compute stream (RCCL's
            # stream waits on it), reduce the staging slice
            st = self.stage[b.start:b.end]
            _cast_scale(buf, st, 1.0 / self.world)
            buf = st
            self._staged = True
        if self._serial and self._works:
            self._works[-1].wait()
        w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._works.append(w)
        self._work_bucket.append(i)

    def _cast_back(self):
        g, st = self.flat.grads, self.stage
        if g.is_cuda:
            from .. import _native
            _native.require_hip().cast_f32_bf16(st, g)
        else:
            g.copy_(st)


def _flush_reductions(buf_device):
    if buf_device.type == "cuda":
        from ..ops import flush_deferred
        flush_deferred()


def _cast_scale(src: torch.Tensor, dst: torch.Tensor, scale: float):
    if src.is_cuda:
        from .. import _native
        _native.require_hip().cast_scale_bf16_f32(src, dst, scale)
    else:
        torch.mul(src.float(), scale, out=dst)


def broadcast_buffers(tensors, src: int = 0, group=None):
    """Broadcast many small non-arena tensors (BatchNorm running stats, step
    counters) in one collective per dtype instead of one each.

    On the GPU the pack/unpack is a single HIP launch each way
    (``flatten_scale``, csrc/hip/bucket.hip); ResNet-50's 106 fp32 BN stats
    become one RCCL broadcast at job start.  Other dtypes (the int64
    ``num_batches_tracked``) go through torch.cat / copy_."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dt, ts in by_dtype.items():
        n = sum(t.numel() for t in ts)
        flat = torch.empty(n, dtype=dt, device=ts[0].device)
        offs, o = [], 0
        for t in ts:
            offs.append(o)
            o += t.numel()
        hip = ts[0].is_cuda and dt in (torch.float32, torch.bfloat16) and all(t.is_contiguous() for t in ts)
        if hip:
            from .. import _native
            m = _native.require_hip()
            m.flatten_scale(ts, flat, offs, 1.0, False)
        else:
            torch.cat([t.reshape(-1) for t in ts], out=flat)
        dist.broadcast(flat, src, group=group)
        if hip:
            m.flatten_scale(ts, flat, offs, 1.0, True)
        else:
            for t, off in zip(ts, offs):
                t.copy_(flat[off:off + t.numel()].view_as(t))
