"""Shared machinery of the HIP op bindings (``ops.gpt2``, ``ops.resnet``).

* device dispatch (``use_hip``): a GPU tensor runs the HIP kernel in
  ``csrc/hip`` — a missing extension raises, never a silent fallback;
* plain PyTorch fp32 references (``ref_*``): the CPU path and the numerics
  tests' oracle (``tests/test_ops_gpu.py``);
* the flat-arena gradient hand-off: weight / bias / norm-weight gradients
  written or reduced straight into the parameter's arena slice
  (``_arena_grads``, ``_signal_ready``), deferred batched column sums
  (``deferred_reductions``), the step's prebuilt Wᵀ operands (``transpose``);
* ``linear`` on gemm_nt4 (forward, dX) and gemm_dw4 (dW into the arena).

The module-level one-element lists (``_NT_ALL``, ``_HIP_DW``, …) are test
hooks that switch a fused path off for an on/off comparison; they are not
user knobs (round 5 retired the ``PDO_*`` environment switches that set them).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from .. import _native


def use_hip(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    if _native.ops_mode() == "torch":
        return False
    _native.require_hip()
    return True

# ----------------------------------------------------------------------------
# reference implementations (fp32 math, cast back to input dtype)
# ----------------------------------------------------------------------------

def ref_layer_norm(x, w, b, eps=1e-5):
    y = F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(x.dtype)


def _gelu_tanh(x):
    return 0.5 * x * (1.0 + torch.tanh(0.7978845608028654 * (x + 0.044715 * x * x * x)))


def ref_bias_gelu(x, b):
    return _gelu_tanh(x.float() + b.float()).to(x.dtype)


def ref_attention(q, k, v, causal=True):
    """q,k,v: [B, H, S, D] → [B, H, S, D] (fp32 math)."""
    qf, kf, vf = q.float(), k.float(), v.float()
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        S = q.shape[-2]
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return (p @ vf).to(q.dtype)


def ref_cross_entropy(logits, target, vocab: int | None = None):
    """Mean token cross entropy; columns >= ``vocab`` (padding) are masked."""
    lf = logits.float()
    if vocab is not None and vocab < lf.shape[-1]:
        lf = lf[..., :vocab]
    return F.cross_entropy(lf.reshape(-1, lf.shape[-1]), target.reshape(-1))


# ----------------------------------------------------------------------------
# linear with direct-to-arena weight gradient
# ----------------------------------------------------------------------------

class _LinearFn(torch.autograd.Function):
    """y = x W^T (+ b) on the hand-written gemm_nt (csrc/hip/gemm_nt4.hip, bias
    fused in the register epilogue) where its shape contract holds.

    Backward: dX on gemm_nt (as F.linear(dY, Wᵀ)), dW on gemm_dw4 written
    straight into the parameter's slice of the flat gradient arena (no
    separate gradient tensor, no AccumulateGrad add kernel), then the bucketed
    all-reduce is signalled that the parameter is ready.  The bias gradient is
    a HIP column reduction."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        ctx.b = b
        return _fwd_gemm(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        K = x.shape[-1]
        Fo = dy.shape[-1]
        dy2 = dy.reshape(-1, Fo)
        x2 = x.reshape(-1, K)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _input_grad(dy2, w).view(x.shape)
        dw = _weight_grad(w, dy2, x2) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            if use_hip(dy2):
                gd = _arena_grads((ctx.b,))
                db = _native.require_hip().bias_grad(dy2.contiguous(), out=gd[0] if gd else None)
                if gd is not None:
                    _signal_ready((ctx.b,))
                    db = None
            else:
                db = dy2.float().sum(0).to(dy.dtype)
        return dx, dw, db


_WS = {}


def _workspace(device, numel):
    """Grow-only bf16 scratch per device (split-K partials)."""
    buf = _WS.get(device)
    if buf is None or buf.numel() < numel:
        buf = torch.empty(numel, dtype=torch.bfloat16, device=device)
        _WS[device] = buf
    return buf[:numel]


def _splitk(tokens: int, m: int, n: int) -> int:
    """Token-slice count for dW = dY^T X: aim for ≥256 output tiles of 256² (one per CU).

    The LM-head dW (50304×1024 → 786 tiles, K = 65536) is past that target but
    still runs 6-8 % faster as 4 token slices (tools/dw_probe.py, tuned).
    Padding the vocabulary to 50432 so gemm_dw takes it measured 6.10 ms (4
    slices) vs 6.35 ms here (tools/lm_dw_probe.py): not worth untuned
    forward / dX shapes for 0.16 % of the step."""
    if tokens < 8192:
        return 1
    tiles = max(1, (m * n) // 65536)
    if 256 <= tiles < 2048:
        return 4 if tokens >= 32768 and tokens % 4 == 0 else 1
    s = 1
    while s < 8 and tiles * s < 256 and tokens % (2 * s) == 0 and tokens // (2 * s) >= 2048:
        s *= 2
    return s


_DX_TN = [True]

# Every forward-layout GEMM (y = x·Wᵀ (+ b): QKV / proj / fc2 forward, the
# input-gradient GEMMs as F.linear(dY, Wᵀ), the LM head) on the hand-written
# gemm_nt4 instead of hipBLASLt, where its shape contract holds (M, N % 256,
# K % 128, or N % 256 = 128 like the 50304-column LM head).  Default since the
# row-accumulator schedules (profiles/r3_gemm_nt4_rows.md): no hipBLASLt kernel
# in the step.  (Test hook: 0 keeps the library for the GEMMs without a fused
# epilogue, 1 routes all of them, any larger value routes those with K ≤ it.)
_NT_ALL = [1]


def _fwd_gemm(x, w, b=None):
    """F.linear(x, w, b) — on gemm_nt4 under _NT_ALL when the shapes allow."""
    if (_NT_ALL[0] and (_NT_ALL[0] == 1 or x.shape[-1] <= _NT_ALL[0])
            and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.is_contiguous() and w.is_contiguous() and (b is None or b.dtype == torch.bfloat16)):
        x2 = x.reshape(-1, x.shape[-1])
        m = _native.require_hip()
        if m.gemm_nt_supported(x2.shape[0], w.shape[0], w.shape[1]):
            return m.gemm_nt(x2, w, b).view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, b)


def _input_grad(dy2, w):
    """dX = dY·W as the forward's GEMM form F.linear(dY, Wᵀ) on gemm_nt.

    gemm_nt reads both operands K-contiguous; the explicit Wᵀ copy is ≤ 8 M
    elements per projection and runs in the LDS-tiled HIP transpose
    (csrc/hip/transpose.hip) at the HBM rate."""
    if _DX_TN[0] and dy2.is_cuda:
        return _fwd_gemm(dy2, transpose(w))
    return dy2 @ w


def _live_wt(w):
    """The arena's prebuilt Wᵀ of ``w`` (parallel.flat.FlatParams.enable_wt) while
    it is live (inside the trainer's wt_scope), else None."""
    t = getattr(w, "_pdo_wt", None)
    if t is not None and t[0].wt_live:
        return t[1]
    return None


def _transposable(w) -> bool:
    return (w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and w.shape[0] % 64 == 0
            and w.shape[1] % 64 == 0 and w.is_contiguous())


def transpose(w, out=None):
    """Contiguous Wᵀ of a 2-D tensor (HIP kernel for bf16 with 64-multiple dims).

    (Measured, round 3: the step's 97 transposes prefetched on a side stream
    under the forward GEMMs made the step 1 ms slower — 148.2 vs 147.2 ms,
    profiles/r3_attention_variants_a5.md — so they stay in-stream.)"""
    if out is None:
        wt = _live_wt(w)
        if wt is not None:
            return wt
    if _transposable(w):
        if out is not None:
            return _native.require_hip().transpose(w, out)
        return _native.require_hip().transpose(w)
    return w.t().contiguous()


def _weight_grad(w, dy2, x2):
    """dW = dy2ᵀ·x2.  Straight into the flat arena when the parameter allows it
    (returns None), else as a tensor for autograd to accumulate.

    (A/B on 1×MI355X: issuing these GEMMs on a side HIP stream to overlap the
    memory-bound backward kernels gained nothing — 394.5k vs 394.7k tok/s — and
    stalled one run on cross-stream allocator reuse; they stay in-stream.)"""
    Fo, K = dy2.shape[1], x2.shape[1]
    if not _direct_ok(w):
        # a gradient tensor for autograd to accumulate (the tied LM head / embedding
        # weight): HIP dW GEMM where its shape contract holds (incl. the 50304-row
        # vocabulary's half-height tile row: 5.42 vs 6.41 ms alone, tools/lm_dw_probe.py;
        # in the step 159.08 / 159.20 vs 159.24 / 159.44 ms, tools/gpu.sh soab)
        if (_HIP_DW[0] and dy2.is_cuda and dy2.dtype == torch.bfloat16 and dy2.is_contiguous()
                and x2.is_contiguous()):
            g = torch.empty(Fo, K, device=dy2.device, dtype=dy2.dtype)
            if _native.require_hip().gemm_dw(dy2, x2, g, False):
                return g
        s = _splitk(dy2.shape[0], Fo, K) if use_hip(dy2) else 1
        if s == 1:
            return dy2.t() @ x2
        T = dy2.shape[0] // s
        part = torch.bmm(dy2.view(s, T, Fo).transpose(1, 2), x2.view(s, T, K),
                         out=_workspace(dy2.device, s * Fo * K).view(s, Fo, K))
        g = torch.empty(Fo, K, device=dy2.device, dtype=dy2.dtype)
        _native.require_hip().splitk_add(part, g, False)
        return g
    if not (_HIP_DW[0] and dy2.is_cuda and w.grad.dtype == torch.bfloat16 and dy2.is_contiguous()
            and x2.is_contiguous() and _native.require_hip().gemm_dw(dy2, x2, w.grad, True)):
        _weight_grad_lib(w, dy2, x2)
    w._pdo_ready(w)
    return None


# dW on the HIP token-major GEMM (csrc/hip/gemm_dw.hip) where its shape
# contract holds (M, N % 256, tokens % 64); hipBLASLt otherwise.  Measured at
# the GPT-2-medium B=64 shapes (tools/dw_probe.py --pdo-only): qkv 375 vs 390 µs,
# proj 131 vs 160, fc1 462 vs 505, fc2 468 vs 506 (hipBLASLt tuned + HIP fold).
_HIP_DW = [True]


def _weight_grad_lib(w, dy2, x2):
    """Arena dW on hipBLASLt: batched token-slice GEMM + HIP fold, or addmm_."""
    Fo, K = dy2.shape[1], x2.shape[1]
    g = w.grad.view(Fo, K)
    s = _splitk(dy2.shape[0], Fo, K)
    if s > 1:
        # long-K / few-tile dW: batched GEMM over token slices + fused fold into the arena
        T = dy2.shape[0] // s
        part = torch.bmm(dy2.view(s, T, Fo).transpose(1, 2), x2.view(s, T, K),
                         out=_workspace(dy2.device, s * Fo * K).view(s, Fo, K))
        _native.require_hip().splitk_add(part, g, True)
    else:
        g.addmm_(dy2.t(), x2)


def _direct_ok(p) -> bool:
    g = p.grad
    return (getattr(p, "_pdo_direct", False) and g is not None and g.is_contiguous()
            and torch.is_grad_enabled() is False)


def _arena_grads(params):
    """The parameters' arena gradient slices when every one of them takes a
    direct write (bf16 flat arena, see parallel.flat), else None.  Kernels that
    reduce a parameter gradient (LayerNorm γ/β, biases) then accumulate straight
    into the arena — no gradient tensor, no AccumulateGrad add kernel."""
    out = []
    for p in params:
        if p is None or not _direct_ok(p) or p.grad.dtype != torch.bfloat16:
            return None
        out.append(p.grad.view(-1))
    return out


class deferred_reductions:
    """Scope (the trainer's backward) in which the bias / norm-weight gradient
    column sums that kernels reduce into the arena are queued and run in a few
    batched launches (``flush_deferred``: before each bucket all-reduce, and on
    exit) — csrc/hip/bind.cpp colsum_or_defer."""

    def __init__(self, device):
        self.on = torch.device(device).type == "cuda" and _native.ops_mode() != "torch"
        self.prev = False

    def __enter__(self):
        if self.on:
            self.prev = _native.require_hip().colsum_defer(True)
        return self

    def __exit__(self, *exc):
        if self.on:
            _native.require_hip().colsum_defer(self.prev)  # off: flushes the queue


def flush_deferred():
    """Run the queued column sums now (stream-ordered; a no-op when none)."""
    m = _native.hip_ext()
    if m is not None and m.colsum_pending():
        m.colsum_flush()


def _signal_ready(params):
    for p in params:
        p._pdo_ready(p)


def linear(x, w, b=None):
    if use_hip(x):
        return _LinearFn.apply(x, w, b)
    return F.linear(x, w, b)


