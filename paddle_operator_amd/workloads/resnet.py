"""ResNet-50 data-parallel training step (collective mode).

Every convolution runs on the hand-written kernels (``ops.resnet``); MIOpen
serves only the framework reference path (``PDO_OPS=torch``).  For that path
the find results measured once on an MI355X ship in
``paddle_operator_amd/tuning/miopen`` and are installed when the trainer is
built in torch mode (utils.tuning.use_shipped_miopen_db): the default find
mode would otherwise benchmark every convolution config on first use (65 s
before the first step at batch 256).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from ..models.resnet import resnet18_like_tiny, resnet50
from ..parallel.ddp import BucketedDDP, broadcast_buffers
from ..parallel.flat import FlatParams


class FlatSGD:
    """Momentum SGD over the flat fp32 arena: one fused HIP pass on the GPU
    (csrc/hip/optim.hip sgd_flat), the reference's bulk ops on CPU."""

    def __init__(self, flat: FlatParams, lr=0.1, momentum=0.9, weight_decay=5e-5):
        self.flat, self.lr, self.mom, self.wd = flat, lr, momentum, weight_decay
        self.buf = torch.zeros_like(flat.params)
        self.decay = flat.decay_chunks.repeat_interleave(flat.numel // flat.decay_chunks.numel())
        self.step_count = 0

    @torch.no_grad()
    def step(self, grad_scale=1.0):
        g = self.flat.param_grads
        if g.is_cuda and g.dtype == torch.float32:
            from .. import _native
            _native.require_hip().sgd_flat(self.flat.params, g, self.buf, self.flat.decay_chunks, self.lr, self.mom,
                                           self.wd, grad_scale)
            self.step_count += 1
            return
        if grad_scale != 1.0:
            g.mul_(grad_scale)
        g.addcmul_(self.decay, self.flat.params, value=self.wd)
        self.buf.mul_(self.mom).add_(g)
        self.flat.params.add_(self.buf, alpha=-self.lr)
        self.step_count += 1

    def state_dict(self):
        return {"buf": self.buf, "step": self.step_count}

    def load_state_dict(self, sd):
        self.buf.copy_(sd["buf"])
        self.step_count = int(sd["step"])


class ResNetTrainer:
    """``graph=True``: after two eager warm-up steps the whole training step
    (weight cast, forward, loss, backward, SGD update) is captured once into a
    HIP graph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and every later
    ``step()`` is one graph launch behind a fresh draw of the synthetic batch
    into the captured input buffers.  Single-rank only: with the bucketed
    all-reduce enabled the step stays eager (RCCL collectives on the overlap
    stream are not captured)."""

    def __init__(self, batch: int, device, tiny: bool = False, bucket_mb: int = 25, channels_last: bool = True,
                 graph: bool = False):
        from .. import _native
        if _native.ops_mode() == "torch":  # the framework reference path: MIOpen convolutions
            from ..utils.tuning import use_shipped_miopen_db
            use_shipped_miopen_db()
        self.device = torch.device(device)
        self.B = batch
        self.tiny = tiny
        model = (resnet18_like_tiny() if tiny else resnet50()).to(self.device)
        self.cl = channels_last and self.device.type == "cuda"
        if self.cl:
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        self.flat = FlatParams(model, dtype=torch.float32, device=self.device, bucket_bytes=bucket_mb << 20)
        if self.device.type == "cuda" and os.environ.get("PDO_WEIGHT_SHADOW", "1") != "0":
            self.flat.enable_shadow(torch.bfloat16)
        self.ddp = BucketedDDP(self.flat)
        self.opt = FlatSGD(self.flat)
        self.res = 32 if tiny else 224
        self.classes = 10 if tiny else 1000
        self.gen = torch.Generator(device=self.device).manual_seed(dist.get_rank() if dist.is_initialized() else 0)
        self.graph = bool(graph) and self.device.type == "cuda" and not self.ddp.enabled
        self._graph = None  # (CUDAGraph, x buffer (NHWC), x view, labels, loss) once captured
        self._eager_steps = 0

    def sync_initial_weights(self):
        self.ddp.broadcast_params(0)
        if self.ddp.world > 1:
            broadcast_buffers(list(self.model.buffers()), 0)

    def _batch_buffers(self):
        if self.cl:  # drawn in NHWC memory order: a channels_last tensor without a layout copy
            # (bf16: the stem convolution runs in bf16 under autocast anyway — no cast pass)
            xb = torch.empty(self.B, self.res, self.res, 3, device=self.device, dtype=torch.bfloat16)
            x = xb.permute(0, 3, 1, 2)
        else:
            xb = x = torch.empty(self.B, 3, self.res, self.res, device=self.device)
        return xb, x, torch.empty(self.B, device=self.device, dtype=torch.long)

    def _draw(self, xb, yb):
        xb.normal_(generator=self.gen)
        yb.random_(0, self.classes, generator=self.gen)

    def batch(self):
        xb, x, y = self._batch_buffers()
        self._draw(xb, y)
        return x, y

    def step(self):
        """One training step; returns the loss tensor (in graph mode the captured
        loss buffer, overwritten by the next step)."""
        if self._graph is not None:
            g, xb, _, yb, loss = self._graph
            self._draw(xb, yb)
            g.replay()
            self.opt.step_count += 1
            return loss
        if self.graph and self._eager_steps >= 2:
            return self._capture()
        self._eager_steps += 1
        x, y = self.batch()
        return self._step(x, y)

    def _capture(self):
        """Capture one training step on a side stream (the allocator's graph pool
        holds every tensor the step allocates), then run it: the first graph step."""
        xb, x, yb = self._batch_buffers()
        cur = torch.cuda.current_stream(self.device)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            # thread_local: a process group's watchdog thread queries its events
            # while this thread captures (global mode would fail those calls)
            with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
                loss = self._step(x, yb)
        cur.wait_stream(side)
        self.opt.step_count -= 1  # recorded, not run
        self._graph = (g, xb, x, yb, loss)
        return self.step()

    def _step(self, x, y):
        self.flat.zero_grad()
        self.ddp.prepare()
        # bf16 copies of the fp32 master weights: one cast of the arena per step
        with self.flat.shadow_scope(), torch.autocast(self.device.type, dtype=torch.bfloat16,
                                                      enabled=self.device.type == "cuda"):
            out = self.model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        self.ddp.finish()
        self.opt.step(self.ddp.grad_scale)
        # detached: a caller holding the loss must not keep this step's autograd
        # graph (and its AccumulateGrad nodes, bound to this step's stream) alive
        # into the next step — that breaks the graph capture of the third step
        return loss.detach()

    def state_dict(self):
        return {"params": self.flat.params, "opt_buf": self.opt.buf, "buffers": {k: v for k, v in
                                                                                  self.model.named_buffers()}}

    def load_state_dict(self, sd):
        self.flat.params.copy_(sd["params"].to(self.flat.params.device))
        self.opt.buf.copy_(sd["opt_buf"].to(self.opt.buf.device))
        bufs = dict(self.model.named_buffers())
        for k, v in sd.get("buffers", {}).items():
            if k in bufs:
                bufs[k].copy_(v.to(bufs[k].device))
