"""GPT-2 ops on the HIP kernels: LayerNorm (+ residual add / fused residual
GEMM epilogue), the MLP with GELU / GELU′ in gemm_nt4 epilogues, causal flash
attention with the fused QKV-bias gradient, the LM head + cross-entropy, the
token + position embedding.  Each op: HIP path for GPU tensors, PyTorch
reference on CPU (``ops.core``)."""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from .. import _native
from .core import (_HIP_DW, _arena_grads, _direct_ok, _fwd_gemm, _input_grad, _signal_ready, _weight_grad,
                   linear, ref_attention, ref_cross_entropy, transpose, use_hip)

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


def layer_norm_res(x, w, b, eps=1e-5):
    """(x, LN(x)) for a residual-stream tensor that also continues past the
    LayerNorm (GPT-2's embedding output feeding block 0): x is returned as an
    alias (_LNResFn), so its downstream gradient joins the LayerNorm backward in
    one kernel instead of a separate [tokens, C] add."""
    if use_hip(x) and x.is_contiguous():
        return _LNResFn.apply(x, w, b, None, eps)
    return x, layer_norm(x, w, b, eps)


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


_RES_EPI = [True]


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

    With ``_NT_GD`` (default) the fc1 epilogue stores gelu'(hp + b1) instead of
    hp (EPI 7: the derivative shares the GELU's exp2 / rcp) and fc2's input
    gradient is one multiply per element (EPI 8) instead of recomputing the
    derivative with the matrix pipe idle.

    ``res``/``b2`` (optional): the fc2 GEMM also adds its bias and the residual
    stream in the epilogue (gemm_nt4 EPI 5), returning x_res + m + b2 for a
    one-input LayerNorm (_LNResFn, which takes b2's gradient); the residual's
    gradient is dy itself."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2=None, res=None):
        m = _native.require_hip()
        x2 = x.reshape(-1, x.shape[-1])
        ctx.saved_grad = _NT_GD[0] and bool(m.gemm_nt_epi_ok(x2.shape[0], w1.shape[0], w1.shape[1]))
        hp, h = m.gemm_nt_gelu(x2, w1, b1, saved_grad=ctx.saved_grad)  # hp = gelu'(x·W1ᵀ + b1) when saved_grad
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
            (dhp,) = m.gemm_nt_dgelu(dy2, transpose(w2), hp, b1, db_out=gd[0], saved_grad=ctx.saved_grad)
            _signal_ready((b1,))
            db1 = None
        else:
            dhp, db1 = m.gemm_nt_dgelu(dy2, transpose(w2), hp, b1, saved_grad=ctx.saved_grad)
        dw1 = _weight_grad(w1, dhp, x2) if ctx.needs_input_grad[1] else None  # its bucket can go first
        dx = _input_grad(dhp, w1).view(ctx.shape) if ctx.needs_input_grad[0] else None
        return dx, dw1, db1, dw2, None, (dy if ctx.res else None)


# fc1 forward with the fused GELU epilogue (gemm_nt): on by default since the
# three-barrier gemm_nt4 schedule (round 3).  GPT-2-medium step, one box, 2
# interleaved rounds (tools/gpu.sh 'stepab:...', profiles/r3_gemm_nt4_sched.md):
# 151.02 / 151.14 ms with hipBLASLt + bias_gelu_fwd, 150.76 / 150.79 fused.
# (Round 2, on the one-barrier schedule, it was 0.5 ms slower: off then.)
# (Test hook: False restores the library GEMM + the HIP bias-GELU kernel.)
_NT_GELU = [True]


# fc2 input gradient with the fused GELU' epilogue (gemm_nt) where its shape
# contract holds; False (test hook) restores hipBLASLt + the bias-GELU kernel.
_NT_DGELU = [True]

# _NTMLPFn saves gelu' from the fc1 epilogue (EPI 7 / 8) instead of the
# pre-activation (−0.8 ms/step, profiles/r5gd_saved_gelu_grad.md); False (test hook) =
# the recomputing pair (EPI 2 / 3), kept under tests/test_ops_gpu.py
_NT_GD = [True]


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


_QKV_FUSED = [True]


def qkv_attention(h: torch.Tensor, w: torch.Tensor, b: torch.Tensor, n_head: int) -> torch.Tensor:
    """attention(linear(h, w, b)) — fused QKV-bias gradient on the HIP path
    (``_QKV_FUSED`` off: separate linear + attention nodes)."""
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
    The chunk is ``_LM_CHUNK`` tokens (``lm_head_xent``): 16384 caps the
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
        # part (bucket 0 launches after the last of them: AuxGrad.node_done), and a
        # forward whose graph is dropped leaves the slot untouched
        sp = getattr(w, "_pdo_split", None)
        ctx.split = sp
        if sp is not None:
            sp.node_begin()  # the slot is ready once every such node's backward has added (flat.AuxGrad)
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
            sp.node_done()
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
        sp.node_begin()
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
        sp.node_done()
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


# the LM-head token chunk: the chunked LM head + cross-entropy (_LMHeadXentFn); -1
# (default) = one chunk of every token: the LM head, the one-kernel cross-entropy
# (xent_fused) and the dX / dW GEMMs in the forward, dloss applied to dX / dW in the
# backward — 143.55 vs 144.04 ms/step against the separate linear + cross_entropy
# Functions (0), whose statistics and dlogits passes read the 6.6 GB logits twice
# (profiles/r3_xent_fused.md); 16384 caps the logits buffer at 1.6 GB (memory option)
_LM_CHUNK = [int(os.environ.get("PDO_LM_CHUNK", "-1"))]
# the chunk path's cross-entropy as one kernel per row (xent_fused: statistics +
# dlogits, one HBM read of the logits) instead of xent_fwd + xent_bwd (two)
_XENT_FUSED = [True]


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


