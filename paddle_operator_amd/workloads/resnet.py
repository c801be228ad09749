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
    def __init__(self, batch: int, device, tiny: bool = False, bucket_mb: int = 25, channels_last: bool = True):
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
        self._graph, self._warm = None, 0
        self._graphed = (self.device.type == "cuda" and self.ddp.world == 1 and not tiny
                         and _native.ops_mode() == "hip" and os.environ.get("PDO_RESNET_GRAPH", "1") != "0")
        self._side = torch.cuda.Stream(self.device) if self._graphed else None

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

    def _body(self, x, y, cache=True):
        self.flat.zero_grad()
        self.ddp.prepare()
        # bf16 copies of the fp32 master weights: one cast of the arena per step
        with self.flat.shadow_scope(), torch.autocast(self.device.type, dtype=torch.bfloat16,
                                                      enabled=self.device.type == "cuda", cache_enabled=cache):
            out = self.model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        self.ddp.finish()
        self.opt.step(self.ddp.grad_scale)
        return loss

    def step(self):
        if self.graphed:
            return self._graph_step()
        x, y = self.batch()
        return self._body(x, y)

    # ---- whole-step HIP graph (one rank) ----
    # The ResNet-50 step is ~580 kernels; launched one by one the GPU idles
    # between short ones (≈0.8 ms per step at batch 256).  Every tensor the step
    # touches is static (flat arena, shadow, optimizer state, workspaces from the
    # graph's private pool), so the forward, backward and SGD update are captured
    # once and replayed; only the batch is drawn outside, into static buffers.
    # Multi-rank steps stay eager (the bucket all-reduces are issued from
    # autograd hooks).  PDO_RESNET_GRAPH=0 disables it.
    @property
    def graphed(self):
        return self._graphed

    def _graph_step(self):
        if self._graph is None:
            if self._warm < 2:
                # the first two steps run eagerly on a side stream (lazy init and the
                # allocator settle before capture, as torch requires)
                self._warm += 1
                x, y = self.batch()
                side = self._side
                side.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(side):
                    loss = self._body(x, y, cache=False)
                torch.cuda.current_stream(self.device).wait_stream(side)
                return loss
            self._capture()
        self._fill_batch()
        self._graph.replay()
        self.opt.step_count += 1
        return self._g_loss

    def _fill_batch(self):
        self._draw(self._xbuf, self._ybuf)

    def _capture(self):
        self._xbuf, self._x, self._ybuf = self._batch_buffers()
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        step0 = self.opt.step_count
        with torch.cuda.graph(g):
            self._g_loss = self._body(self._x, self._ybuf, cache=False)
        self.opt.step_count = step0
        self._graph = g

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
