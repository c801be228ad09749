"""Flat parameter / gradient arena.

MI355X-first replacement for per-tensor optimizer state and DDP's bucket
copies (the reference operator delegates all of this to the Paddle image,
SURVEY §2.4 "GPU collectives — no call site in the reference"):

* every parameter of the model becomes a view into ONE contiguous buffer in
  the compute dtype (bf16); every ``.grad`` is a view into ONE contiguous grad
  buffer, so an all-reduce bucket is just a slice — no flatten/unflatten copy;
* fp32 master weights and Adam moments are flat buffers of the same layout,
  updated by a single fused HIP kernel (``ops.optim.adamw_``) that also folds in
  the 1/world gradient average and global-norm clipping without a host sync;
* parameters are laid out in *expected gradient-ready order* (reverse
  registration order, tied weights last) so bucket k is ready before bucket
  k+1 and the all-reduce of bucket k overlaps the backward of the layers below;
* every parameter starts on a ``ALIGN``-element boundary (2 KiB in bf16): 16-B
  vector loads are always aligned and the per-chunk weight-decay table needs
  one float per ``ALIGN`` elements;
* ``split`` names (the tied ``wte``): the parameter's gradient has two
  producers far apart in the backward — the LM head (first node of the
  backward) and the embedding (last).  The LM-head part gets its own gradient
  slot (``AuxGrad``) that is bucket 0 of the ready order, so its all-reduce
  overlaps the whole backward; only the embedding part stays in the last
  bucket.  ``fold_split()`` adds the reduced head part into the parameter's
  gradient and zeroes the slot.  The slot sits AFTER the parameter range of
  the gradient buffer: ``params`` / the optimizer state / checkpoints cover
  only ``[0, numel)`` and are the same with or without a split
  (``param_grads`` is the optimizer's view of the gradients).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch
import torch.nn as nn

ALIGN = 1024


@dataclass
class Slot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    shape: torch.Size
    decay: bool


@dataclass
class Bucket:
    index: int
    start: int  # element offset into the flat buffers
    end: int
    slots: list = field(default_factory=list)

    @property
    def numel(self):
        return self.end - self.start


def _round_up(x, m):
    return (x + m - 1) // m * m


def _noop_ready(p):
    return None


class AuxGrad:
    """Second gradient slot of a ``split`` parameter (see module docstring).

    ``grad`` is its arena view (same shape as the parameter); the op that
    produces this part of the gradient writes (or adds) into it and calls
    ``node_done()`` — BucketedDDP counts it like a parameter of bucket 0.

    Several graph nodes may write the slot in one step (two forwards through
    the LM head before one backward): each forward registers its node
    (``node_begin``) and the slot is reported ready only when the LAST of them
    has added its part.  Reporting at the first would launch bucket 0's
    all-reduce while the second node's add is still to come — RCCL reducing a
    buffer the compute stream then writes.  A node whose graph is dropped never
    ends; its bucket is then launched by ``BucketedDDP.finish`` (stragglers).
    ``BucketedDDP.prepare`` resets the count: call it before the forward."""

    def __init__(self, name: str, grad: torch.Tensor):
        self.name = name
        self.grad = grad
        self.ready = _noop_ready
        self.nodes = 0

    def node_begin(self):
        self.nodes += 1

    def node_done(self):
        self.nodes -= 1
        if self.nodes <= 0:
            self.nodes = 0
            self.ready(self)


def default_no_decay(name: str, p: torch.Tensor) -> bool:
    """Biases, norm weights and 1-D params are not decayed."""
    return p.dim() < 2


class FlatParams:
    """Owns the flat buffers of a model. See module docstring."""

    def __init__(self, model: nn.Module, dtype=torch.bfloat16, device=None,
                 bucket_bytes: int = 64 << 20, late: tuple = (), no_decay=default_no_decay, split: tuple = ()):
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        if not named:
            raise ValueError("model has no trainable parameters")
        device = torch.device(device) if device is not None else named[0][1].device
        # expected gradient-ready order: reverse registration, `late` names last
        order = list(reversed(named))
        late_set = set(late)
        order = [x for x in order if x[0] not in late_set] + [x for x in order if x[0] in late_set]

        self.dtype = dtype
        self.device = device
        self.slots: list[Slot] = []
        # split parameters' second gradient slots first (ready first: bucket 0)
        params = dict(named)
        unknown = set(split) - set(params)
        if unknown:
            raise ValueError(f"split names not among the trainable parameters: {sorted(unknown)}")
        off = 0
        for n, p in order:
            self.slots.append(Slot(n, p, off, p.numel(), p.shape, not no_decay(n, p)))
            off = _round_up(off + p.numel(), ALIGN)
        self.numel = off  # the parameter range: params, optimizer state, checkpoints
        # split parameters' head-gradient slots after the parameter range (bucket 0)
        self.aux_slots: list[Slot] = []
        goff = off
        for n in split:
            p = params[n]
            self.aux_slots.append(Slot(n + "#head", None, goff, p.numel(), p.shape, False))
            goff = _round_up(goff + p.numel(), ALIGN)
        self.params = torch.zeros(off, dtype=dtype, device=device)
        self.grads = torch.zeros(goff, dtype=dtype, device=device)
        self.param_grads = self.grads[:off]
        # keep each parameter's memory format (e.g. channels_last conv weights
        # for MIOpen NHWC kernels): the arena slice is viewed with its strides
        self._strides = {}
        for s in self.slots:
            p = s.param
            dense = p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))
            self._strides[s.name] = tuple(p.stride()) if dense else None
        with torch.no_grad():
            for s in self.slots:
                self._view(self.params, s).copy_(s.param.detach())
        for s in self.slots:
            s.param.data = self._view(self.params, s)
            s.param.grad = self._view(self.grads, s)
            # ops.linear may write dW straight into the arena; parameters used
            # in several places (tied embeddings) keep autograd accumulation
            s.param._pdo_direct = s.name not in late_set
            s.param._pdo_ready = _noop_ready
            s.param._pdo_split = None
        by_name = {s.name: s for s in self.slots}
        for a in self.aux_slots:
            owner = by_name[a.name[:-len("#head")]]
            a.param = AuxGrad(a.name, self._view(self.grads, a))
            owner.param._pdo_split = a.param
        # one weight-decay flag per ALIGN-element chunk
        wd = torch.zeros(off // ALIGN, dtype=torch.float32)
        for s in self.slots:
            if s.decay:
                c0 = s.offset // ALIGN
                c1 = _round_up(s.offset + s.numel, ALIGN) // ALIGN
                wd[c0:c1] = 1.0
        self.decay_chunks = wd.to(device)
        self.buckets = self._make_buckets(bucket_bytes)

    def enable_shadow(self, dtype=torch.bfloat16):
        """A low-precision copy of the whole arena for the compute kernels (fp32
        master weights, bf16 operands): refreshed by ONE cast of the arena per
        forward (shadow_scope) instead of a cast per weight per forward.  Each
        parameter gets ``_pdo_shadow = (arena, view)``; consumers use the view only
        while ``arena.shadow_live`` (inside shadow_scope), so a weight changed
        outside the trainer's step is never read stale."""
        self.shadow = torch.empty(self.numel, dtype=dtype, device=self.device)
        self.shadow_live = False
        for s in self.slots:
            s.param._pdo_shadow = (self, self._view(self.shadow, s))
        # convolution weights (channels_last [K, C, R, S] = OHWI memory) also get their
        # input-gradient operand Wᵀ [C, R·S·K], built for all of them in one launch
        self.shadow_t, self._wt_table, self._wt_max = None, None, 0
        convs = [s for s in self.slots if len(s.shape) == 4 and s.param.is_contiguous(memory_format=torch.channels_last)
                 and s.param.shape[1] % 8 == 0]
        if convs and self.device.type == "cuda":
            self.shadow_t = torch.empty(self.numel, dtype=dtype, device=self.device)
            rows = []
            for s in convs:
                K, C, R, S = s.shape
                rows.append((s.offset, K, R * S, C))
                s.param._pdo_shadow_t = self.shadow_t[s.offset:s.offset + s.numel].view(C, R * S * K)
                self._wt_max = max(self._wt_max, R * S * ((K + 63) // 64) * ((C + 63) // 64))  # 64 × 64 tiles
            self._wt_table = torch.tensor(rows, dtype=torch.int32, device=self.device)

    def enable_wt(self):
        """A transposed copy Wᵀ of every 2-D weight (dims multiples of 64), for the
        input-gradient GEMMs dX = dY·W that run as F.linear(dY, Wᵀ) on gemm_nt:
        built for all of them in ONE launch per step (``wt_scope``) instead of one
        transpose per weight per backward.  Each such parameter gets
        ``_pdo_wt = (arena, Wᵀ view)``, read only while ``arena.wt_live``."""
        rows, tile = [], 0
        for s in self.slots:
            p = s.param
            if len(s.shape) == 2 and s.shape[0] % 64 == 0 and s.shape[1] % 64 == 0 and p.is_contiguous():
                R, C = s.shape
                rows.append((tile, s.offset, s.offset, R, C))
                tile += (R // 64) * (C // 64)
        self.wt, self.wt_live = None, False
        if not rows or self.device.type != "cuda" or self.dtype != torch.bfloat16:
            return
        self.wt = torch.empty(self.numel, dtype=self.dtype, device=self.device)
        self._wt_host = torch.tensor(rows, dtype=torch.int64)
        self._wt_dev = self._wt_host.to(self.device)
        self._wt_tiles = tile
        by_off = {s.offset: s for s in self.slots}
        for (_, off, _, R, C) in rows:
            by_off[off].param._pdo_wt = (self, self.wt[off:off + R * C].view(C, R))

    def wt_scope(self):
        """Build every Wᵀ (one launch) and mark them live for the scope: the
        trainer's forward + backward, where the weights do not change."""
        flat = self

        class _Scope:
            def __enter__(self):
                if getattr(flat, "wt", None) is not None:
                    from .. import _native
                    _native.require_hip().transpose_batched(flat.params, flat.wt, flat._wt_dev, flat._wt_host,
                                                            flat._wt_tiles)
                    flat.wt_live = True

            def __exit__(self, *exc):
                flat.wt_live = False

        return _Scope()

    def shadow_scope(self):
        flat = self

        class _Scope:
            def __enter__(self):
                if getattr(flat, "shadow", None) is not None:
                    flat.shadow.copy_(flat.params)
                    if flat.shadow_t is not None:
                        from .. import _native
                        _native.require_hip().conv_weight_t_batched(flat.shadow, flat.shadow_t, flat._wt_table,
                                                                     flat._wt_max)
                    flat.shadow_live = True

            def __exit__(self, *exc):
                flat.shadow_live = False

        return _Scope()

    def _view(self, buf, s):
        seg = buf[s.offset:s.offset + s.numel]
        st = self._strides.get(s.name)
        return seg.as_strided(s.shape, st) if st is not None else seg.view(s.shape)

    def _make_buckets(self, bucket_bytes):
        esz = torch.empty((), dtype=self.dtype).element_size()
        cap = max(ALIGN, bucket_bytes // esz)
        buckets, cur = [], None
        # the head slots (after the parameter range) never share a bucket with
        # parameters: a bucket is one contiguous slice of the gradient buffer
        for group in (self.aux_slots, self.slots):
            for s in group:
                if cur is None:
                    cur = Bucket(len(buckets), s.offset, s.offset)
                cur.slots.append(s)
                cur.end = _round_up(s.offset + s.numel, ALIGN)
                if cur.numel >= cap:
                    buckets.append(cur)
                    cur = None
            if cur is not None:
                buckets.append(cur)
                cur = None
        return buckets

    def bucket_of(self):
        m = {}
        for b in self.buckets:
            for s in b.slots:
                m[id(s.param)] = b.index
        return m

    def zero_grad(self):
        self.grads.zero_()

    def fold_split(self):
        """Add each split parameter's head slot into its gradient and zero the
        slot (after the all-reduce drain; every micro-step, so gradient
        accumulation under no_sync sums both parts)."""
        for a in self.aux_slots:
            owner = next(s for s in self.slots if s.name == a.name[:-len("#head")])
            g = self._view(self.grads, owner).view(-1)
            h = self.grads[a.offset:a.offset + a.numel]
            if g.is_cuda and g.dtype == torch.bfloat16:
                from .. import _native
                _native.require_hip().fold_zero(g, h)
            else:
                g.add_(h)
                h.zero_()

    def rebind_grads(self):
        """Re-point .grad at the arena (after anything replaced it)."""
        for a in self.aux_slots:
            a.param.grad = self._view(self.grads, a)
        for s in self.slots:
            g = s.param.grad
            view = self._view(self.grads, s)
            if g is None or g.data_ptr() != view.data_ptr():
                if g is not None:
                    view.copy_(g)
                s.param.grad = view

    def state_dict(self):
        return {s.name: s.param.detach() for s in self.slots}

    def legacy_head_elems(self, n: int) -> int:
        """Checkpoints written before the split head-gradient slots moved behind
        the parameter range (round 5) lead with those slots in params / master /
        m / v: a buffer of exactly ``numel + Σ round_up(slot, ALIGN)`` elements is
        that layout, and the leading elements returned here are dropped on load."""
        head = sum(_round_up(a.numel, ALIGN) for a in self.aux_slots)
        return head if head and n == self.numel + head else 0

    def from_checkpoint(self, buf: torch.Tensor) -> torch.Tensor:
        """A checkpointed parameter-range buffer in this arena's layout; raises
        on a buffer of another model."""
        n = buf.numel()
        skip = self.legacy_head_elems(n)
        if n - skip != self.numel:
            raise ValueError(f"checkpoint arena has {n} elements, this model's has {self.numel}: "
                             "saved by a different model or arena layout")
        return buf.reshape(-1)[skip:]

    def load_params(self, flat_params: torch.Tensor):
        """Copy a checkpointed flat parameter buffer into the arena (either
        layout, ``from_checkpoint``); a buffer of another model raises."""
        self.params.copy_(self.from_checkpoint(flat_params).to(self.params.device))
