"""Fused ops for the flagship workloads.

Every op has two implementations:

* the HIP/CDNA4 kernel in ``csrc/hip`` (used for every CUDA/HIP tensor), and
* a plain PyTorch fp32 reference (``ref_*``), used on CPU and as the oracle in
  the numerics tests (``tests/test_ops_gpu.py``).

Dispatch is by device, never by try/except: a GPU tensor with the extension
missing raises (see ``paddle_operator_amd._native.require_hip``).
"""
from __future__ import annotations

import math

import os

import torch
import torch.nn.functional as F

from .. import _native

__all__ = [
    "layer_norm", "add_layer_norm", "bias_gelu", "attention", "cross_entropy",
    "embedding", "ref_layer_norm", "ref_bias_gelu", "ref_attention",
    "ref_cross_entropy", "use_hip",
]


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
# LayerNorm (optionally fused with the residual add)
# ----------------------------------------------------------------------------

class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        m = _native.require_hip()
        x2 = x.reshape(-1, x.shape[-1])
        y, mean, rstd = m.layernorm_fwd(x2, w, b, eps)
        ctx.save_for_backward(x2, w, mean, rstd)
        ctx.shape = x.shape
        ctx.params = (w, b)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        x2, w, mean, rstd = ctx.saved_tensors
        gd = _arena_grads(ctx.params)
        if gd is not None:
            (dx,) = m.layernorm_bwd(dy.reshape(x2.shape).contiguous(), x2, w, mean, rstd, grads=gd)
            _signal_ready(ctx.params)
            return dx.view(ctx.shape), None, None, None
        dx, dw, db = m.layernorm_bwd(dy.reshape(x2.shape).contiguous(), x2, w, mean, rstd)
        return dx.view(ctx.shape), dw, db, None


def layer_norm(x, w, b, eps=1e-5):
    if use_hip(x):
        return _LayerNormFn.apply(x.contiguous(), w, b, eps)
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)


class _AddLayerNormFn(torch.autograd.Function):
    """h = x + r (+ rbias) ; y = LN(h).  Returns (h, y).

    One read of x and r, one write of h and y: the residual stream never makes
    a separate HBM round trip.  ``rbias`` is the bias of the GEMM that produced
    ``r`` (attention / MLP output projection) folded in; its gradient is the
    column sum of dh, reduced inside the LayerNorm backward kernel."""

    @staticmethod
    def forward(ctx, x, r, w, b, rbias, eps):
        m = _native.require_hip()
        x2 = x.reshape(-1, x.shape[-1])
        r2 = r.reshape(-1, r.shape[-1])
        h, y, mean, rstd = m.add_layernorm_fwd(x2, r2, w, b, eps, rbias)
        ctx.save_for_backward(h, w, mean, rstd)
        ctx.shape = x.shape
        ctx.has_rbias = rbias is not None
        ctx.params = (w, b, rbias) if rbias is not None else (w, b)
        return h.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, dh, dy):
        m = _native.require_hip()
        h, w, mean, rstd = ctx.saved_tensors
        gd = _arena_grads(ctx.params)
        outs = m.layernorm_bwd_add(dy.reshape(h.shape).contiguous(), h, w, mean, rstd,
                                   dh.reshape(h.shape).contiguous(), ctx.has_rbias, grads=gd)
        if gd is not None:
            _signal_ready(ctx.params)
            dx = outs[0].view(ctx.shape)
            return dx, dx, None, None, None, None
        dx = outs[0].view(ctx.shape)
        drb = outs[3] if ctx.has_rbias else None
        return dx, dx, outs[1], outs[2], drb, None


def add_layer_norm(x, r, w, b, eps=1e-5, rbias=None):
    if use_hip(x):
        return _AddLayerNormFn.apply(x.contiguous(), r.contiguous(), w, b, rbias, eps)
    h = x + r if rbias is None else x + r + rbias
    return h, F.layer_norm(h, (h.shape[-1],), w, b, eps)


class _LNResFn(torch.autograd.Function):
    """(h, LN(h)) for a residual-stream tensor h that the producing GEMM already
    summed (x + proj(a) + bias in its epilogue, _LinearResFn / _NTMLPFn): the
    LayerNorm reads h once and writes y — no second input read and no h write
    (_AddLayerNormFn's x + r pass).  h is returned as an alias so the
    downstream residual gradient reaches this backward and joins the
    LayerNorm's in one kernel (layernorm_bwd_add), which also reduces the
    gradient of the producer's bias (``rbias``: added in the GEMM, its gradient
    — the column sum of dh — taken here)."""

    @staticmethod
    def forward(ctx, h, w, b, rbias, eps):
        m = _native.require_hip()
        h2 = h.reshape(-1, h.shape[-1])
        y, mean, rstd = m.layernorm_fwd(h2, w, b, eps)
        ctx.save_for_backward(h2, w, mean, rstd)
        ctx.shape = h.shape
        ctx.has_rbias = rbias is not None
        ctx.params = (w, b, rbias) if rbias is not None else (w, b)
        return h, y.view(h.shape)

    @staticmethod
    def backward(ctx, dh, dy):
        m = _native.require_hip()
        h2, w, mean, rstd = ctx.saved_tensors
        gd = _arena_grads(ctx.params)
        dh2 = dh.reshape(h2.shape).contiguous() if dh is not None else torch.zeros_like(h2)
        outs = m.layernorm_bwd_add(dy.reshape(h2.shape).contiguous(), h2, w, mean, rstd, dh2, ctx.has_rbias,
                                   grads=gd)
        dx = outs[0].view(ctx.shape)
        if gd is not None:
            _signal_ready(ctx.params)
            return dx, None, None, None, None
        return dx, outs[1], outs[2], (outs[3] if ctx.has_rbias else None), None


class _LinearResFn(torch.autograd.Function):
    """h = a·Wᵀ + b + x on gemm_nt4's EPI 5 (bias and the residual stream x
    summed in the register epilogue, one rounding).  ``b`` is taken as a
    constant here: its gradient is reduced by the LayerNorm that consumes h
    (_LNResFn's rbias).  Backward: dA, dW as _LinearFn; dx = dh."""

    @staticmethod
    def forward(ctx, a, w, b, x):
        m = _native.require_hip()
        a2 = a.reshape(-1, a.shape[-1])
        h = m.gemm_nt_add(a2, w, x.reshape(-1, x.shape[-1]), bias=b)
        ctx.save_for_backward(a2, w)
        ctx.shape = a.shape
        return h.view(x.shape)

    @staticmethod
    def backward(ctx, dh):
        a2, w = ctx.saved_tensors
        dh2 = dh.reshape(-1, dh.shape[-1]).contiguous()
        da = _input_grad(dh2, w).view(ctx.shape) if ctx.needs_input_grad[0] else None
        dw = _weight_grad(w, dh2, a2) if ctx.needs_input_grad[1] else None
        return da, dw, None, dh


_RES_EPI = [os.environ.get("PDO_RES_EPI", "1") != "0"]


def _res_epi_ok(T, w, x) -> bool:
    """The residual-stream GEMM epilogue applies to [T, K]·Wᵀ → [T, N] + x: bf16
    contiguous operands on the 4-wave gemm_nt4 path (K % 128, K ≥ 256) within
    its shape contract."""
    N, K = w.shape
    if not (_RES_EPI[0] and use_hip(x) and w.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and w.is_contiguous() and x.is_contiguous() and x.numel() == T * N):
        return False
    return K % 128 == 0 and K >= 256 and bool(_native.require_hip().gemm_nt_supported(T, N, K))


def linear_add_layer_norm(a, w, b, x, ln_w, ln_b, eps=1e-5):
    """(h, LN(h)) with h = x + a·Wᵀ + b — GPT-2's attention output projection
    joining the residual stream: the sum in the GEMM epilogue (_LinearResFn)
    and a one-input LayerNorm (_LNResFn) where the shapes allow, else the GEMM
    + the fused add+LayerNorm pass."""
    if (a.is_cuda and a.dtype == torch.bfloat16 and a.is_contiguous()
            and _res_epi_ok(a.numel() // a.shape[-1], w, x)):
        hs = _LinearResFn.apply(a, w, b.detach(), x)
        return _LNResFn.apply(hs, ln_w, ln_b, b, eps)
    return add_layer_norm(x, linear(a, w), ln_w, ln_b, eps, rbias=b)


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
    if tokens < 8192 or os.environ.get("PDO_SPLITK", "1") == "0":
        return 1
    tiles = max(1, (m * n) // 65536)
    if 256 <= tiles < 2048:
        return 4 if tokens >= 32768 and tokens % 4 == 0 else 1
    s = 1
    while s < 8 and tiles * s < 256 and tokens % (2 * s) == 0 and tokens // (2 * s) >= 2048:
        s *= 2
    return s


_DX_TN = [os.environ.get("PDO_DX_TN", "1") != "0"]

# Every forward-layout GEMM (y = x·Wᵀ (+ b): QKV / proj / fc2 forward, the
# input-gradient GEMMs as F.linear(dY, Wᵀ), the LM head) on the hand-written
# gemm_nt4 instead of hipBLASLt, where its shape contract holds (M, N % 256,
# K % 128, or N % 256 = 128 like the 50304-column LM head).  Default since the
# row-accumulator schedules (profiles/r3_gemm_nt4_rows.md): no hipBLASLt kernel
# in the step.  PDO_NT_ALL=0 keeps the library for the GEMMs without a fused
# epilogue, 1 routes all of them, any larger value routes those with K ≤ it.
_NT_ALL = [int(os.environ.get("PDO_NT_ALL", "1"))]


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
_HIP_DW = [os.environ.get("PDO_HIP_DW", "1") != "0"]


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


# ----------------------------------------------------------------------------
# bias + GELU(tanh)
# ----------------------------------------------------------------------------

class _BiasGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b):
        m = _native.require_hip()
        x2 = x.reshape(-1, x.shape[-1])
        y = m.bias_gelu_fwd(x2, b)
        ctx.save_for_backward(x2, b)
        ctx.shape = x.shape
        ctx.bias = b
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        x2, b = ctx.saved_tensors
        gd = _arena_grads((ctx.bias,))
        if gd is not None:
            (dx,) = m.bias_gelu_bwd(dy.reshape(x2.shape).contiguous(), x2, b, db_out=gd[0])
            _signal_ready((ctx.bias,))
            return dx.view(ctx.shape), None
        dx, db = m.bias_gelu_bwd(dy.reshape(x2.shape).contiguous(), x2, b)
        return dx.view(ctx.shape), db


class _GeluLinearFn(torch.autograd.Function):
    """y = gelu(hp + b1)·W2ᵀ, the back half of the GPT-2 MLP.

    Forward is the HIP bias-GELU kernel + gemm_nt.  Backward runs fc2's
    input-gradient GEMM on gemm_nt (csrc/hip/gemm_nt.hip) with the bias-GELU
    backward fused into its epilogue — dhp = (dY·W2) ⊙ gelu'(hp + b1) and the
    b1 gradient from the tile's fp32 column partials — so the [tokens, 4C]
    gradient makes one HBM trip instead of three (GEMM write, read + write).
    Measured at [65536, 1024] → 4096 on 1×MI355X: 694 µs vs 740 µs for
    hipBLASLt + bias_gelu_bwd (tools/nt_probe.py fc2_dx)."""

    @staticmethod
    def forward(ctx, hp, b1, w2):
        m = _native.require_hip()
        hp2 = hp.reshape(-1, hp.shape[-1])
        h = m.bias_gelu_fwd(hp2, b1)
        ctx.save_for_backward(hp2, h, w2)
        ctx.b1 = b1
        ctx.shape = hp.shape
        return _fwd_gemm(h, w2).view(*hp.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        hp2, h, w2 = ctx.saved_tensors
        b1 = ctx.b1
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dw2 = _weight_grad(w2, dy2, h) if ctx.needs_input_grad[2] else None
        w2t = transpose(w2)
        gd = _arena_grads((b1,))
        if gd is not None:
            (dhp,) = m.gemm_nt_dgelu(dy2, w2t, hp2, b1, db_out=gd[0])
            _signal_ready((b1,))
            db1 = None
        else:
            dhp, db1 = m.gemm_nt_dgelu(dy2, w2t, hp2, b1)
        return dhp.view(ctx.shape), db1, dw2


class _NTMLPFn(torch.autograd.Function):
    """m = gelu(x·W1ᵀ + b1)·W2ᵀ with both GELU passes inside gemm_nt epilogues.

    fc1 forward runs gemm_nt's GELU epilogue (csrc/hip/gemm_nt4.hip, EPI 2):
    the tile writes the pre-activation hp (the backward's GELU' input) and
    h = gelu(hp + b1) from registers, so the [tokens, 4C] activation is not
    re-read by a separate bias-GELU pass.  Backward = _GeluLinearFn's fused
    dGELU epilogue plus fc1's dW / dX.  Measured at [65536, 1024] → 4096 on
    1×MI355X: 598.7 µs vs 644.5 µs for hipBLASLt + bias_gelu_fwd
    (tools/nt4_probe.py fc1_fwd, profiles/r2_gemm_nt4.md).

    ``res``/``b2`` (optional): the fc2 GEMM also adds its bias and the residual
    stream in the epilogue (gemm_nt4 EPI 5), returning x_res + m + b2 for a
    one-input LayerNorm (_LNResFn, which takes b2's gradient); the residual's
    gradient is dy itself."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2=None, res=None):
        m = _native.require_hip()
        x2 = x.reshape(-1, x.shape[-1])
        hp, h = m.gemm_nt_gelu(x2, w1, b1)
        ctx.save_for_backward(x2, w1, hp, h, w2)
        ctx.b1 = b1
        ctx.shape = x.shape
        ctx.res = res is not None
        if res is not None:
            return m.gemm_nt_add(h, w2, res.reshape(-1, res.shape[-1]), bias=b2).view(res.shape)
        return _fwd_gemm(h, w2).view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        x2, w1, hp, h, w2 = ctx.saved_tensors
        b1 = ctx.b1
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dw2 = _weight_grad(w2, dy2, h) if ctx.needs_input_grad[3] else None
        gd = _arena_grads((b1,))
        if gd is not None:
            (dhp,) = m.gemm_nt_dgelu(dy2, transpose(w2), hp, b1, db_out=gd[0])
            _signal_ready((b1,))
            db1 = None
        else:
            dhp, db1 = m.gemm_nt_dgelu(dy2, transpose(w2), hp, b1)
        dw1 = _weight_grad(w1, dhp, x2) if ctx.needs_input_grad[1] else None  # its bucket can go first
        dx = _input_grad(dhp, w1).view(ctx.shape) if ctx.needs_input_grad[0] else None
        return dx, dw1, db1, dw2, None, (dy if ctx.res else None)


# fc1 forward with the fused GELU epilogue (gemm_nt): on by default since the
# three-barrier gemm_nt4 schedule (round 3).  GPT-2-medium step, one box, 2
# interleaved rounds (tools/gpu.sh 'stepab:...', profiles/r3_gemm_nt4_sched.md):
# 151.02 / 151.14 ms with hipBLASLt + bias_gelu_fwd, 150.76 / 150.79 fused.
# (Round 2, on the one-barrier schedule, it was 0.5 ms slower: off then.)
# PDO_NT_GELU=0 restores the library GEMM + the HIP bias-GELU kernel.
_NT_GELU = [os.environ.get("PDO_NT_GELU", "1") != "0"]


# fc2 input gradient with the fused GELU' epilogue (gemm_nt) where its shape
# contract holds; PDO_NT_DGELU=0 restores hipBLASLt + the bias-GELU kernel.
_NT_DGELU = [os.environ.get("PDO_NT_DGELU", "1") != "0"]


def _nt_dgelu_ok(hp, w2) -> bool:
    if not (_NT_DGELU[0] and hp.is_cuda and hp.dtype == torch.bfloat16 and hp.is_contiguous()):
        return False
    tokens = hp.numel() // hp.shape[-1]
    return bool(_native.require_hip().gemm_nt_supported(tokens, w2.shape[1], w2.shape[0]))


def mlp(x, w1, b1, w2):
    """GPT-2 MLP branch without the output bias (folded into the next
    add+LayerNorm): both GELU passes inside gemm_nt epilogues (_NTMLPFn) where
    the shapes allow, else the HIP bias-GELU kernels around plain GEMMs."""
    if (_NT_GELU[0] and use_hip(x) and x.dtype == torch.bfloat16 and x.is_contiguous()
            and _nt_dgelu_ok(x, w2)
            and _native.require_hip().gemm_nt_supported(x.numel() // x.shape[-1], w1.shape[0], w1.shape[1])):
        return _NTMLPFn.apply(x, w1, b1, w2, None, None)
    hp = linear(x, w1)
    if use_hip(hp) and _nt_dgelu_ok(hp, w2):
        return _GeluLinearFn.apply(hp, b1, w2)
    return linear(bias_gelu(hp, b1), w2)


def mlp_add_layer_norm(x, w1, b1, w2, b2, res, ln_w, ln_b, eps=1e-5):
    """(h, LN(h)) with h = res + mlp(x) + b2 — GPT-2's MLP output joining the
    residual stream: fc2's GEMM epilogue adds b2 and res (_NTMLPFn with res) and
    the LayerNorm reads h once (_LNResFn) where the shapes allow, else
    mlp() + the fused add+LayerNorm pass."""
    T = x.numel() // x.shape[-1]
    if (_NT_GELU[0] and use_hip(x) and x.dtype == torch.bfloat16 and x.is_contiguous()
            and _nt_dgelu_ok(x, w2) and _native.require_hip().gemm_nt_supported(T, w1.shape[0], w1.shape[1])
            and _res_epi_ok(T, w2, res)):
        hs = _NTMLPFn.apply(x, w1, b1, w2, b2.detach(), res)
        return _LNResFn.apply(hs, ln_w, ln_b, b2, eps)
    return add_layer_norm(res, mlp(x, w1, b1, w2), ln_w, ln_b, eps, rbias=b2)


def bias_gelu(x, b):
    if use_hip(x):
        return _BiasGeluFn.apply(x.contiguous(), b)
    return F.gelu(x + b, approximate="tanh")


# ----------------------------------------------------------------------------
# causal attention, q/k/v packed as produced by the QKV projection
# ----------------------------------------------------------------------------

class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_head):
        # qkv: [B, S, 3, H, D] (the natural output layout of x @ W_qkv)
        m = _native.require_hip()
        o, lse = m.attn_fwd(qkv, n_head)
        ctx.save_for_backward(qkv, o, lse)
        ctx.n_head = n_head
        return o

    @staticmethod
    def backward(ctx, do):
        m = _native.require_hip()
        qkv, o, lse = ctx.saved_tensors
        dqkv = m.attn_bwd(do.contiguous(), qkv, o, lse, ctx.n_head)[0]
        return dqkv, None


class _QKVAttnFn(torch.autograd.Function):
    """o = attention(h·Wᵀ + b): the QKV projection and causal attention as one
    autograd node, so the backward kernels can hand over the QKV bias gradient.

    The attention backward kernels already hold every dq/dk/dv row in
    registers; they also emit fp32 column sums over their 128 rows, reduced
    here into the bias gradient (accumulated straight into the arena).  This
    replaces a separate column-sum pass over the [tokens, 3C] dqkv (67 µs per
    GPT-2-medium layer at B=64)."""

    @staticmethod
    def forward(ctx, h, w, b, n_head):
        m = _native.require_hip()
        h2 = h.reshape(-1, h.shape[-1])
        qkv = _fwd_gemm(h2, w, b).view(*h.shape[:-1], w.shape[0])
        o, lse = m.attn_fwd(qkv, n_head)
        ctx.save_for_backward(h2, w, qkv, o, lse)
        ctx.b = b
        ctx.n_head = n_head
        ctx.shape = h.shape
        return o

    @staticmethod
    def backward(ctx, do):
        m = _native.require_hip()
        h2, w, qkv, o, lse = ctx.saved_tensors
        b = ctx.b
        gd = _arena_grads((b,)) if ctx.needs_input_grad[2] else None
        db = None
        if gd is not None:
            (dqkv,) = m.attn_bwd(do.contiguous(), qkv, o, lse, ctx.n_head, True, gd[0])
            _signal_ready((b,))
        elif ctx.needs_input_grad[2]:
            dqkv, db = m.attn_bwd(do.contiguous(), qkv, o, lse, ctx.n_head, True)
        else:
            (dqkv,) = m.attn_bwd(do.contiguous(), qkv, o, lse, ctx.n_head)
        dq2 = dqkv.view(-1, dqkv.shape[-1])
        dh = _input_grad(dq2, w).view(ctx.shape) if ctx.needs_input_grad[0] else None
        dw = _weight_grad(w, dq2, h2) if ctx.needs_input_grad[1] else None
        return dh, dw, db, None


_QKV_FUSED = [os.environ.get("PDO_QKV_FUSED", "1") != "0"]


def qkv_attention(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, n_head: int) -> torch.Tensor:
    """attention(linear(h, w, b)) — fused QKV-bias gradient on the HIP path
    (PDO_QKV_FUSED=0: separate linear + attention nodes)."""
    S, C3 = h.shape[-2], w.shape[0]
    if _QKV_FUSED[0] and use_hip(h) and b is not None and (C3 // 3) // n_head == 64 and S % 128 == 0 and h.dim() == 3:
        return _QKVAttnFn.apply(h, w, b, n_head)
    return attention(linear(h, w, b), n_head)


def attention(qkv: torch.Tensor, n_head: int) -> torch.Tensor:
    """Causal self-attention.

    ``qkv``: [B, S, 3*C] straight out of the QKV GEMM; returns [B, S, C].
    HIP path: MFMA flash attention reading q/k/v in place (no transposes).
    """
    B, S, C3 = qkv.shape
    C = C3 // 3
    D = C // n_head
    if use_hip(qkv) and D == 64 and S % 128 == 0:
        return _FlashAttnFn.apply(qkv.contiguous(), n_head)
    # shapes outside the hand-written kernel's contract (head_dim != 64 or
    # seq % 128 != 0) use the framework SDPA on GPU / the fp32 reference on CPU
    q, k, v = qkv.view(B, S, 3, n_head, D).permute(2, 0, 3, 1, 4).unbind(0)
    if qkv.is_cuda:
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    else:
        o = ref_attention(q, k, v, causal=True)
    return o.transpose(1, 2).reshape(B, S, C)


# ----------------------------------------------------------------------------
# softmax cross entropy over a (padded) vocabulary
# ----------------------------------------------------------------------------

class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, vocab):
        m = _native.require_hip()
        l2 = logits.reshape(-1, logits.shape[-1])
        t = target.reshape(-1)
        loss, lse, stats = m.xent_fwd(l2, t, vocab)
        ctx.save_for_backward(l2, t, lse, stats)
        ctx.vocab = vocab
        ctx.shape = logits.shape
        return loss.clone()

    @staticmethod
    def backward(ctx, dloss):
        m = _native.require_hip()
        l2, t, lse, stats = ctx.saved_tensors
        # the logits buffer is dead after this point: write dlogits in place
        dl = m.xent_bwd(l2, t, lse, dloss.reshape(1).float().contiguous(), stats, ctx.vocab, True)
        return dl.view(ctx.shape), None, None


class _LMHeadXentFn(torch.autograd.Function):
    """loss = CE(h·Wᵀ, target) with the LM head and the cross-entropy run over
    token chunks: per chunk the logits GEMM (gemm_nt4), the softmax statistics,
    dlogits written in place, the chunk's dX GEMM and its dW GEMM accumulated
    into one [Vp, C] gradient — so only a [chunk, Vp] logits buffer exists.
    The chunk is ``PDO_LM_CHUNK`` tokens (``lm_head_xent``): 16384 caps the
    buffer at 1.6 GB; the default (-1) is one chunk of every token, i.e. the
    whole [tokens, Vp] logits tensor (6.6 GB at GPT-2-medium B = 64), which
    ran 0.5 ms/step faster (profiles/r3_xent_fused.md).  The gradients are
    computed in the forward, for dloss = 1, and applied scaled by dloss in the
    backward (the loss is the graph's last node)."""

    @staticmethod
    def forward(ctx, h, w, target, vocab, chunk):
        m = _native.require_hip()
        h2 = h.reshape(-1, h.shape[-1])
        t = target.reshape(-1)
        N, C = h2.shape
        Vp = w.shape[0]
        wt = transpose(w)
        valid = ((t >= 0) & (t < vocab)).sum().float()
        stats = torch.stack([torch.zeros_like(valid), valid])  # xent_bwd reads the count from stats[1]
        ones = torch.ones(1, device=h.device, dtype=torch.float32)
        fused = _XENT_FUSED[0]
        inv_cnt = (1.0 / valid.clamp(min=1.0)).reshape(1)
        logits = torch.empty(chunk, Vp, device=h.device, dtype=h.dtype)
        dh = torch.empty_like(h2)
        # dW stays private to this node until its backward: a split tied weight
        # (parallel/flat.py) then adds it, scaled by dloss, into its head-gradient
        # slot (bucket 0) — two forwards before one backward each add their own
        # part, and a forward whose graph is dropped leaves the slot untouched
        sp = getattr(w, "_pdo_split", None)
        ctx.split = sp
        dw = torch.empty(Vp, C, device=h.device, dtype=h.dtype)
        loss_sum = torch.zeros((), device=h.device, dtype=torch.float32)
        for c0 in range(0, N, chunk):
            hc, tc = h2[c0:c0 + chunk], t[c0:c0 + chunk]
            lg = logits[:hc.shape[0]]
            m.gemm_nt(hc, w, None, lg)
            if fused:
                # one kernel: row statistics, then (softmax − onehot) / count in place
                # (the chunk's loss already divided by the total count)
                loss_sum += m.xent_fused(lg, tc, inv_cnt, vocab)
                dl = lg
            else:
                _, lse, st = m.xent_fwd(lg, tc, vocab)  # st = (chunk mean loss, chunk valid count)
                loss_sum += st[0] * st[1]
                dl = m.xent_bwd(lg, tc, lse, ones, stats, vocab, True)  # (softmax − onehot) / count, in place
            m.gemm_nt(dl, wt, None, dh[c0:c0 + chunk])
            if not m.gemm_dw(dl, hc, dw, c0 > 0):
                if c0 == 0:
                    dw.copy_(dl.t() @ hc)
                else:
                    dw.addmm_(dl.t(), hc)
        ctx.save_for_backward(dh, dw)
        ctx.shape = h.shape
        return loss_sum if fused else loss_sum / valid

    @staticmethod
    def backward(ctx, dloss):
        dh, dw = ctx.saved_tensors
        # scaled in fp32, rounded once: a non-unit dloss (1/accum_steps) is not
        # first rounded to bf16
        # in place, one pass each: x = bf16(f32(x) · dloss) with dloss read on device
        m = _native.require_hip()
        d = dloss.float().reshape(1).contiguous()
        m.scale_dev_(dh, d)
        sp = ctx.split
        if sp is not None:
            m.axpy_dev_(sp.grad.view(-1), dw.view(-1), d)  # slot += dloss · dW, one rounding
            sp.ready(sp)
            return dh.view(ctx.shape), None, None, None, None
        m.scale_dev_(dw, d)
        return dh.view(ctx.shape), dw, None, None, None


class _SplitHeadLinearFn(torch.autograd.Function):
    """logits = h·Wᵀ for a split tied weight outside _LMHeadXentFn's contract
    (CPU, unsupported shapes): the backward adds dW into the weight's
    head-gradient slot (parallel/flat.py AuxGrad) and signals it ready, instead
    of accumulating into the gradient the embedding also writes."""

    @staticmethod
    def forward(ctx, h, w, sp):
        ctx.save_for_backward(h, w)
        ctx.sp = sp
        return _fwd_gemm(h, w) if h.is_cuda else F.linear(h, w)

    @staticmethod
    def backward(ctx, dy):
        h, w = ctx.saved_tensors
        sp = ctx.sp
        V, C = w.shape
        dy2 = dy.reshape(-1, V)
        h2 = h.reshape(-1, C)
        dh = (_input_grad(dy2.contiguous(), w) if dy.is_cuda else dy2 @ w).view(h.shape)
        g = sp.grad.view(V, C)
        if not (dy.is_cuda and dy2.dtype == torch.bfloat16 and _HIP_DW[0] and dy2.is_contiguous()
                and h2.is_contiguous() and _native.require_hip().gemm_dw(dy2, h2, g, True)):
            g.addmm_(dy2.t().to(g.dtype), h2.to(g.dtype))
        sp.ready(sp)
        return dh, None, None


def _lm_head_loss_only(h, w, target, vocab: int, chunk: int):
    """Loss of the tied LM head without gradients (no_grad / eval): the logits
    GEMM and the statistics pass per chunk — no dX / dW GEMMs, no [Vp, C]
    gradient buffer."""
    m = _native.require_hip()
    h2 = h.reshape(-1, h.shape[-1])
    t = target.reshape(-1)
    N = h2.shape[0]
    logits = torch.empty(min(chunk, N), w.shape[0], device=h.device, dtype=h.dtype)
    loss_sum = torch.zeros((), device=h.device, dtype=torch.float32)
    cnt = torch.zeros((), device=h.device, dtype=torch.float32)
    for c0 in range(0, N, chunk):
        hc, tc = h2[c0:c0 + chunk], t[c0:c0 + chunk]
        lg = logits[:hc.shape[0]]
        m.gemm_nt(hc, w, None, lg)
        _, _, st = m.xent_fwd(lg, tc, vocab)  # (chunk mean loss, chunk valid count)
        loss_sum += st[0] * st[1]
        cnt += st[1]
    return loss_sum / cnt.clamp(min=1.0)


# PDO_LM_CHUNK=tokens: the chunked LM head + cross-entropy (_LMHeadXentFn); -1
# (default) = one chunk of every token: the LM head, the one-kernel cross-entropy
# (xent_fused) and the dX / dW GEMMs in the forward, dloss applied to dX / dW in the
# backward — 143.55 vs 144.04 ms/step against the separate linear + cross_entropy
# Functions (0), whose statistics and dlogits passes read the 6.6 GB logits twice
# (profiles/r3_xent_fused.md); 16384 caps the logits buffer at 1.6 GB (memory option)
_LM_CHUNK = [int(os.environ.get("PDO_LM_CHUNK", "-1"))]
# the chunk path's cross-entropy as one kernel per row (xent_fused: statistics +
# dlogits, one HBM read of the logits) instead of xent_fwd + xent_bwd (two)
_XENT_FUSED = [os.environ.get("PDO_XENT_FUSED", "1") != "0"]


def lm_head_xent(h, w, target, vocab: int):
    """Mean cross-entropy of the tied LM head h·Wᵀ over the first ``vocab`` columns."""
    N = h.numel() // h.shape[-1]
    ch = _LM_CHUNK[0]
    if ch < 0:
        ch = N
    if (ch and use_hip(h) and h.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and N % ch == 0
            and h.is_contiguous() and w.is_contiguous()
            and _native.require_hip().gemm_nt_supported(ch, w.shape[0], w.shape[1])
            and _native.require_hip().gemm_nt_supported(ch, w.shape[1], w.shape[0])):
        if not (torch.is_grad_enabled() and (h.requires_grad or w.requires_grad)):
            return _lm_head_loss_only(h, w, target, vocab, ch)
        return _LMHeadXentFn.apply(h, w, target, vocab, ch)
    sp = getattr(w, "_pdo_split", None)
    if sp is not None and torch.is_grad_enabled() and w.requires_grad:
        return cross_entropy(_SplitHeadLinearFn.apply(h, w, sp), target, vocab)
    return cross_entropy(linear(h, w), target, vocab)


def cross_entropy(logits, target, vocab: int | None = None):
    V = vocab if vocab is not None else logits.shape[-1]
    if use_hip(logits):
        return _XentFn.apply(logits.contiguous(), target.contiguous(), V)
    return ref_cross_entropy(logits, target, V)


# ----------------------------------------------------------------------------
# token + position embedding
# ----------------------------------------------------------------------------

class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe):
        m = _native.require_hip()
        y = m.embed_fwd(idx, wte, wpe)
        ctx.save_for_backward(idx)
        ctx.wte_shape = wte.shape
        ctx.wpe_shape = wpe.shape
        ctx.dtype = wte.dtype
        ctx.wte = wte
        return y

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        (idx,) = ctx.saved_tensors
        wte = ctx.wte
        g = wte.grad
        # split tied weight (parallel/flat.py): the LM head's part of the gradient has
        # its own slot, so the embedding is this slot's only producer — add straight
        # into it (sorted segmented sum, deterministic), no fp32 table, no
        # AccumulateGrad add
        if (getattr(wte, "_pdo_split", None) is not None and g is not None and g.dtype == torch.bfloat16
                and g.is_contiguous() and ctx.dtype == torch.bfloat16 and not torch.is_grad_enabled()):
            keys, perm = torch.sort(idx.reshape(-1), stable=True)
            dwpe = m.embed_bwd_sorted(dy.contiguous(), keys, perm, g, ctx.wpe_shape[0])
            wte._pdo_ready(wte)
            return None, None, dwpe
        dwte, dwpe = m.embed_bwd(dy.contiguous(), idx, ctx.wte_shape[0], ctx.wpe_shape[0])
        return None, dwte.to(ctx.dtype), dwpe.to(ctx.dtype)


def embedding(idx, wte, wpe):
    """y[b, s] = wte[idx[b, s]] + wpe[s]."""
    if use_hip(wte):
        return _EmbedFn.apply(idx.contiguous(), wte, wpe)
    S = idx.shape[1]
    return F.embedding(idx, wte) + wpe[:S].unsqueeze(0)


# ----------------------------------------------------------------------------
# BatchNorm (training) + ReLU (+ residual add) for NHWC bf16 — ResNet-50
# ----------------------------------------------------------------------------

class _BNActFn(torch.autograd.Function):
    """y = act(BN(x) [+ residual]) with batch statistics (csrc/hip/batchnorm.hip).

    Without a residual the backward recomputes the ReLU mask from x, so only
    x (the conv output autograd keeps anyway) and two [C] vectors are saved.
    ``stats``: the producing convolution's per-tile partials (conv.hip), so the
    forward skips its statistics pass over x.  ``link``: a _BNLink through which
    the consuming implicit-GEMM convolution hands back the backward statistics
    it took in its input-gradient epilogue, so the backward skips its
    statistics pass over dy and x too."""

    @staticmethod
    def forward(ctx, x, w, b, residual, running_mean, running_var, eps, momentum, relu, stats=None, tile_rows=0,
                link=None, rlink=None, mlink=None):
        m = _native.require_hip()
        # mask: with a residual under the ReLU, the 1-bit ReLU mask the backward reads
        # instead of the bf16 output (1/16 of the bytes, both backward passes)
        if stats is not None:
            y, mean, invstd, mask = m.bn_act_fwd_tiles(x, stats, tile_rows, residual, w, b, running_mean,
                                                       running_var, eps, momentum, relu)
        else:
            y, mean, invstd, mask = m.bn_act_fwd(x, residual, w, b, running_mean, running_var, eps, momentum, relu)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, mask if (relu and ctx.has_res) else None, mean, invstd, w, b)
        ctx.params = (w, b)
        ctx.link = link
        if link is not None:
            link.bn = (x, mean, invstd, w, b, relu)
        # residual = a forked convolution input (identity block): its gradient's
        # ReLU mask is applied by that convolution's dX epilogue (_ResMaskLink)
        ctx.rlink = rlink if (rlink is not None and relu and residual is not None and mask is not None) else None
        # this output is another BatchNorm's residual (ResNet's downsample branch): that
        # BatchNorm may hand over (its dy, its ReLU mask) instead of writing dy ⊙ mask
        ctx.mlink = mlink if (mlink is not None and not relu and residual is None) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        x, y, mean, invstd, w, b = ctx.saved_tensors
        pw, pb = ctx.params
        # gamma/beta gradients straight into the flat arena when allowed
        direct = _direct_ok(pw) and _direct_ok(pb) and pw.grad.dtype == torch.float32
        dwi, dbi = (pw.grad, pb.grad) if direct else (None, None)
        part = ctx.link.take(dy) if ctx.link is not None else None
        want_dres = ctx.has_res and ctx.rlink is None
        relu = ctx.relu
        gmask = ctx.mlink.take(dy) if ctx.mlink is not None else None
        ctx.mlink = None
        if gmask is not None:  # dy ⊙ gmask is this BatchNorm's output gradient: the bitmask mode (y = mask)
            y, relu = gmask, True
        if part is not None:
            dx, dres, dw, db = m.bn_act_bwd_part(part, dy, y, x, mean, invstd, w, b, relu, want_dres, dwi, dbi)
        else:
            dx, dres, dw, db = m.bn_act_bwd(dy, y, x, mean, invstd, w, b, relu, want_dres, dwi, dbi)
        ctx.link = None
        if ctx.rlink is not None:
            dres = dy  # unmasked: the forking convolution's dX epilogue applies the mask
            ctx.rlink.give(dy, y)
            ctx.rlink = None
        if direct:
            pw._pdo_ready(pw)
            pb._pdo_ready(pb)
            dw = db = None
        return dx, dw, db, (dres if ctx.has_res else None), None, None, None, None, None, None, None, None, None, None


class _BNLink:
    """Hand-off between a BatchNorm(+ReLU) output and the implicit-GEMM
    convolution that consumes it (ResNet's bn1 → conv2).  Forward: the
    BatchNorm leaves (x, mean, invstd, w, b, relu) here; backward: the
    convolution's input gradient computes, in its epilogue, that BatchNorm's
    Σg and Σg·(x − mean) per tile (conv_dgrad_bn) and parks them with the
    gradient tensor they belong to.  The BatchNorm uses them only when the dy
    it receives IS that tensor, unmodified (same storage and version — another
    consumer's gradient added to it would show as a new tensor or a version
    bump; the reference held here stops autograd from accumulating in place)."""

    __slots__ = ("bn", "dx", "ver", "part")

    def __init__(self):
        self.bn = self.dx = self.part = None
        self.ver = -1

    def give(self, dx, part):
        self.dx, self.ver, self.part = dx, dx._version, part

    def take(self, dy):
        dx, part, ver = self.dx, self.part, self.ver
        self.bn = self.dx = self.part = None
        if (part is None or dy.data_ptr() != dx.data_ptr() or dy._version != ver or dy.shape != dx.shape
                or not dy.is_contiguous(memory_format=torch.channels_last)):
            return None
        _BN_LINK_USED[0] += 1
        return part


_BN_LINK_USED = [0]  # backward passes that took their statistics from a convolution epilogue (tests)

class _ResMaskLink:
    """Hand-off for a residual branch that is a convolution's forked input
    (ResNet's identity block: bn3's residual is the x conv1 forked).  The
    residual BatchNorm's backward does not write dres = dy ⊙ relu-mask: it
    returns dy itself as the residual's gradient and parks (dy, mask) here; the
    forking convolution's input-gradient GEMM applies the mask to that addend in
    its epilogue (gemm_nt_add EPI 6).  A gradient arriving there that is not
    that exact tensor (storage and version) would mean something else was added
    to it — an error, raised, never silently masked."""

    __slots__ = ("dy", "ver", "mask")

    def __init__(self):
        self.dy = self.mask = None
        self.ver = -1

    def give(self, dy, mask):
        self.dy, self.ver, self.mask = dy, dy._version, mask

    def take(self, dalias):
        dy, ver, mask = self.dy, self.ver, self.mask
        self.dy = self.mask = None
        if mask is None:
            return None
        if dalias is None or dalias.data_ptr() != dy.data_ptr() or dalias._version != ver:
            raise RuntimeError("residual mask hand-off: the forked input's gradient is not the residual "
                               "BatchNorm's dy (another consumer added to it)")
        _RES_MASK_USED[0] += 1
        return mask


_RES_MASK_USED = [0]  # identity-branch gradients masked in the conv1 dX epilogue (tests)

class _CompactGradLink:
    """Hand-off from a 1×1 stride-2 convolution (ResNet's downsample) to the
    convolution that forked its input (conv1): the downsample's input gradient is
    nonzero only at the stride-2 pixels, so it is computed compact ([N, C, Ho, Wo],
    one GEMM) and added into conv1's dX at those pixels (conv_stride2_add) instead
    of a zero-filled full-resolution tensor that conv1's GEMM re-reads as its
    addend.  The downsample returns no input gradient through autograd; any other
    gradient of the forked input still arrives as conv1's dalias and is added."""

    __slots__ = ("t",)

    def __init__(self):
        self.t = None

    def give(self, t):
        self.t = t if self.t is None else self.t + t

    def take(self):
        t, self.t = self.t, None
        if t is not None:
            _DS_COMPACT_USED[0] += 1
        return t


_DS_COMPACT_USED = [0]
_DS_COMPACT = [os.environ.get("PDO_DS_COMPACT", "1") != "0"]
_RES_MASK = [os.environ.get("PDO_RES_MASK", "1") != "0"]


def _apply_bitmask(t, mask):
    """t ⊙ keep for a channels_last tensor and its [N·H·W·C / 8] ReLU bitmask."""
    bits = ((mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1).view(-1)
    flat = t.permute(0, 2, 3, 1).reshape(-1) * bits.to(t.dtype)
    return flat.view(t.shape[0], t.shape[2], t.shape[3], t.shape[1]).permute(0, 3, 1, 2)


_BN_FUSED = [os.environ.get("PDO_BN_FUSED", "1") != "0"]
_BN_LINK = [os.environ.get("PDO_BN_LINK", "1") != "0"]


def bn_act(bn: torch.nn.BatchNorm2d, x, relu: bool = True, residual=None, rlink=None, mlink=None):
    """Training BatchNorm → (+ residual) → ReLU in one HIP forward pass over the
    activation (plus a statistics pass), and one backward pass (plus stats).
    Falls back to PyTorch ops outside the fused case (eval mode, CPU, NCHW,
    C % 8 != 0)."""
    fused = (_BN_FUSED[0] and use_hip(x) and bn.training and x.dtype == torch.bfloat16 and x.dim() == 4
             and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0
             and bn.weight is not None and bn.weight.dtype == torch.float32
             and (residual is None or (residual.dtype == torch.bfloat16
                                       and residual.is_contiguous(memory_format=torch.channels_last))))
    if fused:
        mom = bn.momentum if bn.momentum is not None else 0.1
        link = _BNLink() if residual is None and _BN_LINK[0] and torch.is_grad_enabled() else None
        y = _BNActFn.apply(x, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var, bn.eps, mom, relu,
                           None, 0, link, rlink, mlink)
        if link is not None:
            y._pdo_bn = link  # read by _ConvFn when y feeds an implicit-GEMM convolution
        if mlink is not None and not relu and residual is None:
            y._pdo_rlink = mlink  # read by the BatchNorm this output is the residual of
        return y
    y = bn(x)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def _gemm_fwd_1x1(m, T, C, K) -> bool:
    """1×1 stride-1 forward on the token-major GEMM (gemm_nt) rather than the
    implicit GEMM: measured faster for every ResNet-50 shape with K > 128 output
    channels; at K ≤ 128 the implicit GEMM is as fast or faster and its epilogue
    also yields the BatchNorm statistics (profiles/r4d_conv_probe.jsonl)."""
    return K > 128 and bool(m.gemm_nt_supported(T, K, C))


def _gemm_dgrad_1x1(m, T, C, K) -> bool:
    """1×1 stride-1 input gradient on gemm_nt: faster at C > 128 input channels
    (profiles/r4d_conv_probe.jsonl)."""
    return C > 128 and bool(m.gemm_nt_supported(T, C, K))


def _gemm_wgrad_1x1(C, K) -> bool:
    """1×1 stride-1 weight gradient on gemm_dw4 where it has ≥ 8 output tiles
    (1024/2048-channel shapes); conv_wgrad elsewhere."""
    return ((K + 255) // 256) * (C // 256) >= 8


class _ConvFn(torch.autograd.Function):
    """y = conv2d(x, w) for a channels_last bf16 activation on hand-written
    kernels: the NHWC implicit GEMM (csrc/hip/conv.hip) for 3×3 stride 1 / 2 and
    1×1 stride 1 / 2 — forward (+ BatchNorm tile statistics, a second
    non-differentiable output), input gradient (Wᵀ built per backward, stride-2
    parity classes), weight gradient (split-K, fp32, straight into the flat fp32
    arena when the parameter allows it) — and, per product where measured
    faster, the token-major GEMMs for 1×1 stride 1 (gemm_nt / gemm_dw4).

    ``fork``: also return x itself (an autograd alias) for a second consumer —
    ResNet's identity / downsample branch — so that branch's gradient reaches
    this backward and joins dX in the dX kernel's epilogue (no separate add of
    two activation-sized gradients).  Replaces MIOpen's igemm fwd / bwd / wrw
    solvers, their zero-fill / cast passes and the hipBLASLt small-shape weight
    gradients on ResNet-50 (profiles/r3t_resnet50_kernels.md)."""

    @staticmethod
    def forward(ctx, x, w, stride, pad, want_stats, fork=False, rlink=None, slink=None, clink=None):
        m = _native.require_hip()
        sh = getattr(w, "_pdo_shadow", None)  # the arena's bf16 copy, cast once per step (FlatParams.shadow_scope)
        ctx.wt = None
        if sh is not None and sh[0].shadow_live and sh[1].dtype == torch.bfloat16 \
                and sh[1].is_contiguous(memory_format=torch.channels_last):
            wb = sh[1]
            ctx.wt = getattr(w, "_pdo_shadow_t", None)  # Wᵀ, built with the shadow (one launch per step)
        else:
            wb = w.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        K, C, R, _ = wb.shape
        N, _, H, W_ = x.shape
        ctx.one = R == 1 and stride == 1
        st = None
        if ctx.one and _gemm_fwd_1x1(m, N * H * W_, C, K):
            y = m.gemm_nt(x.permute(0, 2, 3, 1).reshape(-1, C), wb.view(K, C)).view(N, H, W_, K).permute(0, 3, 1, 2)
        else:
            y, st = m.conv_fwd(x, wb, stride, pad, want_stats)
        ctx.save_for_backward(x, wb)
        ctx.stride, ctx.pad = stride, pad
        ctx.wparam = w
        link = getattr(x, "_pdo_bn", None)
        ctx.link = link if link is not None and link.bn is not None else None
        ctx.rlink = rlink if fork else None
        ctx.slink = slink if fork else None  # conv1: compact downsample gradients to add into dX
        ctx.clink = clink if (R == 1 and stride == 2 and pad == 0) else None  # downsample: give dX compact
        ctx.set_materialize_grads(False)
        if st is not None:
            ctx.mark_non_differentiable(st)
        return y, st, (x if fork else None)

    @staticmethod
    def backward(ctx, dy, _dstats, dalias):
        m = _native.require_hip()
        x, wb = ctx.saved_tensors
        K, C, R, S = wb.shape
        N, _, H, W_ = x.shape
        T = N * H * W_
        link, ctx.link = ctx.link, None
        rlink, ctx.rlink = ctx.rlink, None
        slink, ctx.slink = ctx.slink, None
        clink, ctx.clink = ctx.clink, None
        amask = rlink.take(dalias) if rlink is not None else None  # dalias ⊙ amask is the branch's gradient
        if dy is None:  # y unused: only the alias carried a gradient
            cadd = slink.take() if slink is not None else None
            if cadd is not None:  # (y unused) the forked input's gradient = dalias + the compact downsample part
                base = (_apply_bitmask(dalias, amask) if amask is not None else dalias)
                base = (base.contiguous(memory_format=torch.channels_last).clone() if base is not None else
                        torch.zeros(ctx.saved_tensors[0].shape, device=cadd.device,
                                    dtype=cadd.dtype).contiguous(memory_format=torch.channels_last))
                m.conv_stride2_add(base, cadd.contiguous(memory_format=torch.channels_last))
                return base, None, None, None, None, None, None, None, None
            return ((_apply_bitmask(dalias, amask) if amask is not None else dalias), None, None, None, None, None, None,
                    None, None)
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dalias is not None:
            dalias = dalias.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0] and clink is not None and dalias is None:
            # the downsample's dX, compact: [N·Ho·Wo, K] · W [K, C] on gemm_nt, for the forking conv1
            No, _, Ho, Wo = dy.shape
            T4 = No * Ho * Wo
            if m.gemm_nt_supported(T4, C, K):
                g = m.gemm_nt(dy.permute(0, 2, 3, 1).reshape(T4, K), transpose(wb.view(K, C)))
                clink.give(g.view(No, Ho, Wo, C).permute(0, 3, 1, 2))
                clink = "given"
        if ctx.needs_input_grad[0] and clink != "given":
            # the GEMM where it is faster, even past a BatchNorm link (that
            # BatchNorm then takes its own statistics pass)
            if ctx.one and _gemm_dgrad_1x1(m, T, C, K):
                dy2 = dy.permute(0, 2, 3, 1).reshape(T, K)
                wt2 = transpose(wb.view(K, C))
                dx = (m.gemm_nt_add(dy2, wt2, dalias.permute(0, 2, 3, 1).reshape(T, C), mask=amask)
                      if dalias is not None else m.gemm_nt(dy2, wt2))
                amask = None
                dx = dx.view(N, H, W_, C).permute(0, 3, 1, 2)
            else:
                if amask is not None:
                    dalias, amask = _apply_bitmask(dalias, amask).contiguous(memory_format=torch.channels_last), None
                wt = ctx.wt if ctx.wt is not None else m.conv_weight_t(wb)
                if link is not None and link.bn is not None:
                    # the producing BatchNorm's backward statistics from this epilogue
                    bx, mean, invstd, bw, bb, relu = link.bn
                    dx, part = m.conv_dgrad_bn(dy, wt, R, S, ctx.stride, ctx.pad, bx, mean, invstd, bw, bb, relu)
                    link.give(dx, part)
                    if dalias is not None:  # (not a ResNet pattern: a BatchNorm output is not forked)
                        dx = dx + dalias
                else:
                    dx = m.conv_dgrad(dy, wt, C, R, S, H, W_, ctx.stride, ctx.pad, dalias)
        cadd = slink.take() if slink is not None else None
        if cadd is not None and dx is not None:
            dx = dx.contiguous(memory_format=torch.channels_last)
            m.conv_stride2_add(dx, cadd.contiguous(memory_format=torch.channels_last))
        if ctx.needs_input_grad[1]:
            p = ctx.wparam
            if ctx.one and _gemm_wgrad_1x1(C, K):
                g = torch.empty(K, C, device=x.device, dtype=torch.bfloat16)
                m.gemm_dw(dy.permute(0, 2, 3, 1).reshape(T, K), x.permute(0, 2, 3, 1).reshape(T, C), g, False)
                dw = g.view(K, C, 1, 1).to(p.dtype)
            elif (_direct_ok(p) and p.grad.dtype == torch.float32
                    and p.grad.is_contiguous(memory_format=torch.channels_last)):
                m.conv_wgrad(dy, x, R, S, ctx.stride, ctx.pad, out=p.grad)
                p._pdo_ready(p)
            else:
                dw = m.conv_wgrad(dy, x, R, S, ctx.stride, ctx.pad).to(p.dtype)
        return dx, dw, None, None, None, None, None, None, None


_HIP_CONV = [os.environ.get("PDO_HIP_CONV", "1") != "0"]


def _hip_conv_ok(conv: torch.nn.Conv2d, x) -> bool:
    if not (_HIP_CONV[0] and use_hip(x) and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and conv.groups == 1 and conv.bias is None
            and conv.dilation == (1, 1) and conv.kernel_size[0] == conv.kernel_size[1]
            and conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]):
        return False
    R, st, pad = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    N, C, H, W = x.shape
    return bool(_native.require_hip().conv_ok(N, H, W, C, conv.out_channels, R, R, st, pad))


def conv1x1(conv: torch.nn.Conv2d, x):
    """``conv(x)`` for a 1×1 bias-free convolution: the hand-written kernels
    (_ConvFn: implicit GEMM or token-major GEMM per product) for channels_last
    bf16 activations on the HIP path, else the framework convolution."""
    if _hip_conv_ok(conv, x):
        return _ConvFn.apply(x, conv.weight, conv.stride[0], conv.padding[0], False)[0]
    return conv(x)


class _StemFn(torch.autograd.Function):
    """ResNet's 7×7 / stride-2 / pad-3 stem convolution (3 → 64 channels) for a
    channels_last bf16 image, as a space-to-depth 4×4 stride-1 convolution over a
    16-channel image (csrc/hip/conv.hip, stem_*): forward on the implicit GEMM
    with the BatchNorm tile statistics in its epilogue, weight gradient on the
    tap-group kernel (dY staged once for the four kernel rows).  The image needs
    no gradient.  Replaces MIOpen's igemm fwd / wrw solvers on 3-channel input
    (≈ 360 µs each at batch 256, profiles/r4p_resnet50_kernels.md)."""

    @staticmethod
    def forward(ctx, x, w):
        m = _native.require_hip()
        sh = getattr(w, "_pdo_shadow", None)
        if sh is not None and sh[0].shadow_live and sh[1].dtype == torch.bfloat16 \
                and sh[1].is_contiguous(memory_format=torch.channels_last):
            wb = sh[1]
        else:
            wb = w.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y, st, z = m.stem_fwd(x, wb, True)
        ctx.save_for_backward(z)
        ctx.wparam = w
        ctx.mark_non_differentiable(st)
        return y, st

    @staticmethod
    def backward(ctx, dy, _dstats):
        m = _native.require_hip()
        (z,) = ctx.saved_tensors
        p = ctx.wparam
        dw = None
        if dy is not None and ctx.needs_input_grad[1]:
            dy = dy.contiguous(memory_format=torch.channels_last)
            if _direct_ok(p) and p.grad.dtype == torch.float32 and p.grad.is_contiguous(memory_format=torch.channels_last):
                m.stem_wgrad(dy, z, p.grad)
                p._pdo_ready(p)
            else:
                dw = m.stem_wgrad(dy, z).to(p.dtype)
        return None, dw


_HIP_STEM = [os.environ.get("PDO_HIP_STEM", "1") != "0"]


def _stem_ok(conv: torch.nn.Conv2d, x) -> bool:
    if not (_HIP_CONV[0] and _HIP_STEM[0] and use_hip(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and not x.requires_grad
            and x.is_contiguous(memory_format=torch.channels_last) and conv.groups == 1 and conv.bias is None
            and conv.dilation == (1, 1) and tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2)
            and tuple(conv.padding) == (3, 3)):
        return False
    N, C, H, W = x.shape
    return bool(_native.require_hip().stem_ok(N, H, W, C, conv.out_channels))


def _bn_fused_ok(bn: torch.nn.BatchNorm2d, residual) -> bool:
    return (bn.training and _BN_FUSED[0] and bn.weight is not None and bn.weight.dtype == torch.float32
            and (residual is None or (residual.dtype == torch.bfloat16
                                      and residual.is_contiguous(memory_format=torch.channels_last))))


def conv_bn_act(conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, x, relu: bool = True, residual=None,
                fork: bool = False, as_residual: bool = False):
    """see _conv_bn_act.  ``residual`` may be a forked input whose only consumer
    besides the forking convolution is this BatchNorm (ResNet's identity
    block): then its ReLU-masked gradient is formed in the forking
    convolution's dX epilogue.  ``as_residual``: the output's only consumer is
    another BatchNorm's residual (ResNet's downsample branch): that BatchNorm
    hands over (dy, ReLU mask) and this backward applies the mask itself."""
    return _conv_bn_act(conv, bn, x, relu, residual, fork, as_residual)


def _conv_bn_act(conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, x, relu: bool = True, residual=None,
                 fork: bool = False, as_residual: bool = False):
    """act(BN(conv(x)) [+ residual]) — on the hand-written convolutions with the
    BatchNorm statistics taken in the implicit GEMM's epilogue where that kernel
    runs the forward; otherwise the framework convolution + ops.bn_act.
    ``fork``: returns (out, x_alias) — x for a second consumer whose gradient
    then joins this convolution's dX in its epilogue (_ConvFn)."""
    stem = not fork and _stem_ok(conv, x)
    if (stem or _hip_conv_ok(conv, x)) and _bn_fused_ok(bn, residual):
        rl = _ResMaskLink() if (fork and _RES_MASK[0] and torch.is_grad_enabled()) else None
        # compact downsample gradients: not past a BatchNorm link (its partials come from dX's epilogue)
        sl = (_CompactGradLink() if (fork and _DS_COMPACT[0] and torch.is_grad_enabled()
                                      and getattr(x, "_pdo_bn", None) is None) else None)
        cl = getattr(x, "_pdo_slink", None) if not fork else None
        if stem:
            y, st = _StemFn.apply(x, conv.weight)
            xa = None
        else:
            y, st, xa = _ConvFn.apply(x, conv.weight, conv.stride[0], conv.padding[0], True, fork, rl, sl, cl)
            if rl is not None and xa is not None:
                xa._pdo_rlink = rl  # read by the residual BatchNorm when xa is its residual
            if sl is not None and xa is not None:
                xa._pdo_slink = sl  # read by a 1×1 stride-2 convolution of xa (the downsample)
        rres = getattr(residual, "_pdo_rlink", None) if residual is not None else None
        ml = (_ResMaskLink() if as_residual and not relu and residual is None and _RES_MASK[0]
              and torch.is_grad_enabled() else None)
        if st is None:
            out = bn_act(bn, y, relu=relu, residual=residual, rlink=rres, mlink=ml)
        else:
            mom = bn.momentum if bn.momentum is not None else 0.1
            m = _native.require_hip()
            rows = m.stem_tile_rows() if stem else m.conv_tile_rows(conv.out_channels)
            link = _BNLink() if residual is None and _BN_LINK[0] and torch.is_grad_enabled() else None
            out = _BNActFn.apply(y, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var, bn.eps, mom,
                                 relu, st, rows, link, rres, ml)
            if link is not None:
                out._pdo_bn = link
            if ml is not None:
                out._pdo_rlink = ml  # read by the BatchNorm this output is the residual of
        return (out, xa) if fork else out
    out = bn_act(bn, conv(x), relu=relu, residual=residual)
    return (out, x) if fork else out


class _BNReluPoolFn(torch.autograd.Function):
    """max_pool_3x3s2(ReLU(BN(x))) for ResNet's stem in one forward pass (from the
    stem convolution's tile statistics) and a two-pass backward
    (csrc/hip/batchnorm.hip bn_relu_pool_* / pool_bn_*): the full-resolution
    activation (256 × 64 × 112 × 112 at batch 256, 411 MB) is neither written
    nor re-read, and its gradient is never materialised — only the BatchNorm
    input gradient the stem's weight gradient reads.  The backward statistics
    run over the pooled tensors (dy, y and the BatchNorm input at each window
    maximum, ``xsel``): a gradient reaches no other pixel."""

    @staticmethod
    def forward(ctx, x, w, b, running_mean, running_var, eps, momentum, stats, tile_rows):
        m = _native.require_hip()
        y, arg, xsel, mean, invstd = m.bn_relu_pool_fwd_tiles(x, stats, tile_rows, w, b, running_mean, running_var,
                                                              eps, momentum)
        ctx.save_for_backward(x, y, xsel, arg, mean, invstd, w, b)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        x, y, xsel, arg, mean, invstd, w, b = ctx.saved_tensors
        pw, pb = ctx.params
        direct = _direct_ok(pw) and _direct_ok(pb) and pw.grad.dtype == torch.float32
        dwi, dbi = (pw.grad, pb.grad) if direct else (None, None)
        dx, dw, db = m.pool_bn_bwd(dy.contiguous(memory_format=torch.channels_last), y, xsel, arg, x, mean, invstd,
                                   w, b, dwi, dbi)
        if direct:
            pw._pdo_ready(pw)
            pb._pdo_ready(pb)
            dw = db = None
        return dx, dw, db, None, None, None, None, None, None


_STEM_POOL = [os.environ.get("PDO_STEM_POOL", "1") != "0"]


def conv_bn_relu_maxpool(conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, x):
    """ResNet stem: max_pool_3x3s2(ReLU(BN(conv(x)))) — the space-to-depth stem
    convolution (_StemFn) with the BatchNorm, ReLU and max-pool fused into one
    pass each way (_BNReluPoolFn) on the HIP path; else conv_bn_act + max-pool."""
    if _STEM_POOL[0] and _stem_ok(conv, x) and _bn_fused_ok(bn, None):
        y, st = _StemFn.apply(x, conv.weight)
        mom = bn.momentum if bn.momentum is not None else 0.1
        return _BNReluPoolFn.apply(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, mom, st,
                                   _native.require_hip().stem_tile_rows())
    return max_pool_3x3s2(conv_bn_act(conv, bn, x))


class _MaxPool3s2Fn(torch.autograd.Function):
    """3×3 / stride 2 / pad 1 max-pool, NHWC bf16 (csrc/hip/pool.hip)."""

    @staticmethod
    def forward(ctx, x):
        y, arg = _native.require_hip().maxpool3s2_fwd(x)
        ctx.save_for_backward(arg)
        ctx.hw = (x.shape[2], x.shape[3])
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        return _native.require_hip().maxpool3s2_bwd(dy, arg, *ctx.hw)


def max_pool_3x3s2(x):
    """ResNet stem pool; HIP gather-backward kernel for channels_last bf16."""
    if (use_hip(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _MaxPool3s2Fn.apply(x)
    return F.max_pool2d(x, 3, 2, 1)
