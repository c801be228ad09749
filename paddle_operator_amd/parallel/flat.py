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
  backward) and the embedding (last).  The LM-head part gets its own arena slot
  at the FRONT of the ready order (``AuxGrad``, bucket 0), so its all-reduce
  overlaps the whole backward; only the embedding part stays in the last
  bucket.  ``fold_split()`` adds the reduced head part into the parameter's
  gradient and zeroes the slot (the optimizer never sees it).
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
    ``ready(self)`` — BucketedDDP counts it like a parameter of bucket 0."""

    def __init__(self, name: str, grad: torch.Tensor):
        self.name = name
        self.grad = grad
        self.ready = _noop_ready


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
        self.aux_slots: list[Slot] = []
        off = 0
        for n in split:
            p = params[n]
            self.aux_slots.append(Slot(n + "#head", None, off, p.numel(), p.shape, False))
            off = _round_up(off + p.numel(), ALIGN)
        for n, p in order:
            self.slots.append(Slot(n, p, off, p.numel(), p.shape, not no_decay(n, p)))
            off = _round_up(off + p.numel(), ALIGN)
        self.numel = off
        self.params = torch.zeros(off, dtype=dtype, device=device)
        self.grads = torch.zeros(off, dtype=dtype, device=device)
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
        for s in self.aux_slots + self.slots:
            if cur is None:
                cur = Bucket(len(buckets), s.offset, s.offset)
            cur.slots.append(s)
            cur.end = _round_up(s.offset + s.numel, ALIGN)
            if cur.numel >= cap:
                buckets.append(cur)
                cur = None
        if cur is not None:
            buckets.append(cur)
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
