"""ResNet-50 ops on the HIP kernels: NHWC implicit-GEMM convolutions with
BatchNorm statistics / residual-gradient epilogues, BatchNorm (+ ReLU,
+ residual) with batch statistics, the space-to-depth stem with its fused
BatchNorm + ReLU + max-pool (``csrc/hip/conv.hip``, ``batchnorm.hip``,
``pool.hip``)."""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import _native
from .core import _arena_grads, _direct_ok, _signal_ready, transpose, use_hip

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
_DS_COMPACT = [True]
_RES_MASK = [True]


def _apply_bitmask(t, mask):
    """t ⊙ keep for a channels_last tensor and its [N·H·W·C / 8] ReLU bitmask."""
    bits = ((mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1).view(-1)
    flat = t.permute(0, 2, 3, 1).reshape(-1) * bits.to(t.dtype)
    return flat.view(t.shape[0], t.shape[2], t.shape[3], t.shape[1]).permute(0, 3, 1, 2)


_BN_FUSED = [True]
_BN_LINK = [True]


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


def _direct_cl_ok(p) -> bool:
    """A convolution weight's fp32 arena gradient takes the kernel's direct
    (accumulating) write: ``_direct_ok`` but for the channels_last [K, C, R, S]
    view the arena keeps for a channels_last weight (``_direct_ok`` asks for the
    NCHW-contiguous layout, which a 3×3 or the stem's 7×7 view is not — those
    went through a temporary and an AccumulateGrad add)."""
    g = p.grad
    return (getattr(p, "_pdo_direct", False) and g is not None and not torch.is_grad_enabled()
            and g.dtype == torch.float32 and g.is_contiguous(memory_format=torch.channels_last))


def _gemm_fwd_1x1(m, T, C, K) -> bool:
    """1×1 stride-1 forward on the token-major GEMM (gemm_nt) rather than the
    implicit GEMM: measured faster for every ResNet-50 shape with K > 128 output
    channels; at K ≤ 128 the implicit GEMM is as fast or faster and its epilogue
    also yields the BatchNorm statistics (profiles/r4d_conv_probe.jsonl)."""
    return K > 128 and bool(m.gemm_nt_supported(T, K, C))


# the 1×1 forward on gemm_nt takes the BatchNorm statistics in its epilogue
# (gemm_nt EPI 9, profiles/r5bs_gemm_bn_stats_epilogue.md); False (test hook) = a
# separate statistics pass over the output
_GEMM_BN_STATS = [True]


def _fwd_stats_rows(m, conv: torch.nn.Conv2d, x) -> int:
    """Rows per partial of the statistics _ConvFn returns for conv(x)."""
    N, C, H, W = x.shape
    if conv.kernel_size[0] == 1 and conv.stride[0] == 1 and _gemm_fwd_1x1(m, N * H * W, C, conv.out_channels):
        return m.gemm_nt_stats_rows(C)
    return m.conv_tile_rows(conv.out_channels)


def _gemm_dgrad_1x1(m, T, C, K) -> bool:
    """1×1 stride-1 input gradient on gemm_nt: faster at C > 128 input channels
    (profiles/r4d_conv_probe.jsonl)."""
    return C > 128 and bool(m.gemm_nt_supported(T, C, K))


def _gemm_wgrad_1x1(C, K) -> bool:
    """1×1 stride-1 weight gradient on gemm_dw4 where it has ≥ 8 output tiles
    (1024/2048-channel shapes); conv_wgrad elsewhere."""
    return ((K + 255) // 256) * (C // 256) >= 8


def _wt_1x1(ctx, wb, K, C):
    """Wᵀ [C, K] of a 1×1 weight for its input-gradient GEMM: the view of the
    step's batched transpose (FlatParams.shadow_t, built with the bf16 shadow in
    one launch) when the forward read the shadow, else one transpose."""
    if ctx.wt is not None and ctx.wt.numel() == C * K:
        return ctx.wt.view(C, K)
    return transpose(wb.view(K, C))


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
            x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
            if want_stats and _GEMM_BN_STATS[0]:
                y, st = m.gemm_nt_stats(x2, wb.view(K, C))  # + BatchNorm partials (EPI 9, _fwd_stats_rows)
            else:
                y = m.gemm_nt(x2, wb.view(K, C))
            y = y.view(N, H, W_, K).permute(0, 3, 1, 2)
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
                g = m.gemm_nt(dy.permute(0, 2, 3, 1).reshape(T4, K), _wt_1x1(ctx, wb, K, C))
                clink.give(g.view(No, Ho, Wo, C).permute(0, 3, 1, 2))
                clink = "given"
        if ctx.needs_input_grad[0] and clink != "given":
            # the GEMM where it is faster, even past a BatchNorm link (that
            # BatchNorm then takes its own statistics pass)
            if ctx.one and _gemm_dgrad_1x1(m, T, C, K):
                dy2 = dy.permute(0, 2, 3, 1).reshape(T, K)
                wt2 = _wt_1x1(ctx, wb, K, C)
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
            g = None
            if ctx.one and _gemm_wgrad_1x1(C, K):
                g = torch.empty(K, C, device=x.device, dtype=torch.bfloat16)
                # False: outside gemm_dw's contract (tokens not a multiple of its
                # 64-token k-tile, e.g. 49·N at layer4 for N % 64 ≠ 0) — g unwritten
                if not m.gemm_dw(dy.permute(0, 2, 3, 1).reshape(T, K), x.permute(0, 2, 3, 1).reshape(T, C), g,
                                 False):
                    g = None
            if g is not None:
                dw = g.view(K, C, 1, 1).to(p.dtype)
            elif _direct_cl_ok(p):
                m.conv_wgrad(dy, x, R, S, ctx.stride, ctx.pad, out=p.grad)
                p._pdo_ready(p)
            else:
                dw = m.conv_wgrad(dy, x, R, S, ctx.stride, ctx.pad).to(p.dtype)
        return dx, dw, None, None, None, None, None, None, None


_HIP_CONV = [True]


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
            if _direct_cl_ok(p):
                m.stem_wgrad(dy, z, p.grad)
                p._pdo_ready(p)
            else:
                dw = m.stem_wgrad(dy, z).to(p.dtype)
        return None, dw


_HIP_STEM = [True]


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
            rows = m.stem_tile_rows() if stem else _fwd_stats_rows(m, conv, x)
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


class _BNActBNResFn(torch.autograd.Function):
    """y = ReLU(BN(x) + BN_r(r)) — ResNet's downsample block tail: bn3 over
    conv3's output x and the downsample BatchNorm over the downsample conv's
    output r, both from their convolutions' tile statistics, in ONE apply pass
    (``bn_act_fwd_tiles_bnres``): the downsample branch's normalised activation
    is never written or re-read.  Backward: each BatchNorm's backward from the
    shared output gradient and ReLU bitmask (what the unfused pair did through
    the residual-mask hand-off) in one statistics and one apply pass over
    (dy, mask, x, r): the shared gradient and mask are read once."""

    @staticmethod
    def forward(ctx, x, w, b, r, rw, rb, rm, rv, eps, mom, rrm, rrv, reps, rmom, stats, rows, rstats, rrows):
        m = _native.require_hip()
        y, mean, invstd, mask, rmean, rinvstd = m.bn_act_fwd_tiles_bnres(
            x, stats, rows, w, b, rm, rv, eps, mom, r, rstats, rrows, rw, rb, rrm, rrv, reps, rmom, True)
        ctx.save_for_backward(x, r, mask, mean, invstd, w, b, rmean, rinvstd, rw, rb)
        ctx.params = (w, b, rw, rb)
        return y

    @staticmethod
    def backward(ctx, dy):
        m = _native.require_hip()
        x, r, mask, mean, invstd, w, b, rmean, rinvstd, rw, rb = ctx.saved_tensors
        into = []
        for pw, pb in (ctx.params[:2], ctx.params[2:]):
            direct = _direct_ok(pw) and _direct_ok(pb) and pw.grad.dtype == torch.float32
            into.append((pw.grad, pb.grad) if direct else (None, None))
        # one statistics pass and one apply pass over (dy, mask, x, r) for both
        dx, dr, dw, db, drw, drb = m.bn_act_bwd_pair(dy, mask, x, mean, invstd, w, r, rmean, rinvstd, rw,
                                                     *into[0], *into[1])
        out = []
        for (pw, pb), (dwi, _), (gw, gb) in zip((ctx.params[:2], ctx.params[2:]), into, ((dw, db), (drw, drb))):
            if dwi is not None:
                pw._pdo_ready(pw)
                pb._pdo_ready(pb)
                gw = gb = None
            out.append((gw, gb))
        (dw, db), (drw, drb) = out
        return dx, dw, db, dr, drw, drb, None, None, None, None, None, None, None, None, None, None, None, None


# ResNet's downsample block: bn3 and the downsample BatchNorm in one apply pass
# (_BNActBNResFn); False = the downsample BatchNorm's own apply pass (A/B, tests)
_DS_FUSED = [True]


def conv_bn_ds_act(conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, x, dconv: torch.nn.Conv2d,
                   dbn: torch.nn.BatchNorm2d, xa):
    """ReLU(BN(conv(x)) + BN_d(dconv(xa))) — a downsample bottleneck's tail.
    Both convolutions on the hand-written kernels with BatchNorm statistics in
    their epilogues, then one apply pass (_BNActBNResFn); otherwise the
    downsample branch through conv_bn_act(as_residual=True) and bn3 with it as
    the residual."""
    m = _native.require_hip() if use_hip(x) else None
    if (m is not None and _DS_FUSED[0] and torch.is_grad_enabled() and _hip_conv_ok(conv, x)
            and _hip_conv_ok(dconv, xa) and _bn_fused_ok(bn, None) and _bn_fused_ok(dbn, None)):
        # the downsample conv first (as the unfused order): its compact input
        # gradient goes to the conv that forked xa (_CompactGradLink)
        cl = getattr(xa, "_pdo_slink", None)
        yd, std, _ = _ConvFn.apply(xa, dconv.weight, dconv.stride[0], dconv.padding[0], True, False, None, None, cl)
        y, st, _ = _ConvFn.apply(x, conv.weight, conv.stride[0], conv.padding[0], True)
        if st is not None and std is not None:
            mom = bn.momentum if bn.momentum is not None else 0.1
            dmom = dbn.momentum if dbn.momentum is not None else 0.1
            return _BNActBNResFn.apply(y, bn.weight, bn.bias, yd, dbn.weight, dbn.bias, bn.running_mean,
                                       bn.running_var, bn.eps, mom, dbn.running_mean, dbn.running_var, dbn.eps, dmom,
                                       st, _fwd_stats_rows(m, conv, x), std, _fwd_stats_rows(m, dconv, xa))
        idt = bn_act(dbn, yd, relu=False)
        return bn_act(bn, y, relu=True, residual=idt)
    idt = conv_bn_act(dconv, dbn, xa, relu=False, as_residual=True)
    return conv_bn_act(conv, bn, x, relu=True, residual=idt)


class _GAPFn(torch.autograd.Function):
    """Global average pool of a channels_last bf16 activation → [N, C]; the
    backward writes dy / HW straight into a channels_last gradient
    (``gap_bwd``) — the framework's broadcast + layout copy of it, and a second
    copy where that gradient was the identity branch's, ran ≈ 0.18 ms per step
    (tools/prof_sequence.py of one ResNet-50 step)."""

    @staticmethod
    def forward(ctx, x):
        ctx.hw = x.shape[2:]
        return x.mean(dim=(2, 3))

    @staticmethod
    def backward(ctx, dy):
        return _native.require_hip().gap_bwd(dy.to(torch.bfloat16).contiguous(), *ctx.hw)


def global_avg_pool(x):
    """``flatten(adaptive_avg_pool2d(x, 1), 1)``; on the HIP path for channels_last bf16."""
    if (use_hip(x) and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last)):
        return _GAPFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


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


_STEM_POOL = [True]


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

