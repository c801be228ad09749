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
  one float per ``ALIGN`` elements.
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


def default_no_decay(name: str, p: torch.Tensor) -> bool:
    """Biases, norm weights and 1-D params are not decayed."""
    return p.dim() < 2


class FlatParams:
    """Owns the flat buffers of a model. See module docstring."""

    def __init__(self, model: nn.Module, dtype=torch.bfloat16, device=None,
                 bucket_bytes: int = 64 << 20, late: tuple = (), no_decay=default_no_decay):
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
        off = 0
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
        # one weight-decay flag per ALIGN-element chunk
        wd = torch.zeros(off // ALIGN, dtype=torch.float32)
        for s in self.slots:
            if s.decay:
                c0 = s.offset // ALIGN
                c1 = _round_up(s.offset + s.numel, ALIGN) // ALIGN
                wd[c0:c1] = 1.0
        self.decay_chunks = wd.to(device)
        self.buckets = self._make_buckets(bucket_bytes)

    def _view(self, buf, s):
        seg = buf[s.offset:s.offset + s.numel]
        st = self._strides.get(s.name)
        return seg.as_strided(s.shape, st) if st is not None else seg.view(s.shape)

    def _make_buckets(self, bucket_bytes):
        esz = torch.empty((), dtype=self.dtype).element_size()
        cap = max(ALIGN, bucket_bytes // esz)
        buckets, cur = [], None
        for s in self.slots:
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

    def rebind_grads(self):
        """Re-point .grad at the arena (after anything replaced it)."""
        for s in self.slots:
            g = s.param.grad
            view = self._view(self.grads, s)
            if g is None or g.data_ptr() != view.data_ptr():
                if g is not None:
                    view.copy_(g)
                s.param.grad = view

    def state_dict(self):
        return {s.name: s.param.detach() for s in self.slots}
