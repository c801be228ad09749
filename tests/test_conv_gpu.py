"""NHWC implicit-GEMM convolutions (csrc/hip/conv.hip) against fp32 PyTorch references.

Shapes are ResNet-50's (3×3 stride 1 / 2, strided 1×1 downsample) at small
batch, plus partial last M-tiles (token count not a multiple of the tile).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from paddle_operator_amd import _native
    return _native.require_hip()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _mk(N, C, H, K, R, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda", generator=g) / (C * R * R) ** 0.5).bfloat16()
    return x, w.contiguous(memory_format=torch.channels_last)


# (N, C, H, K, R, stride): 3×3 s1 (Kout 64 → 256×64 tiles; 128 → 128×128), 3×3 s2, 1×1 s2 downsample,
# H = 7 / 5 with N = 3: token counts that leave a partial last tile
SHAPES = [(2, 64, 16, 64, 3, 1), (2, 128, 14, 128, 3, 1), (2, 128, 16, 128, 3, 2), (3, 64, 7, 128, 3, 1),
          (2, 256, 14, 512, 1, 2), (3, 128, 5, 256, 3, 2), (2, 512, 7, 512, 3, 1)]


@pytest.mark.parametrize("N,C,H,K,R,stride", SHAPES)
def test_conv_fwd_and_tile_stats(hip, N, C, H, K, R, stride):
    x, w = _mk(N, C, H, K, R, 1)
    pad = (R - 1) // 2
    assert hip.conv_ok(N, H, H, C, K, R, R, stride, pad)
    y, st = hip.conv_fwd(x, w, stride, pad, True)
    ref = F.conv2d(x.float(), w.float(), stride=stride, padding=pad)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 1e-2
    # tile statistics reproduce the per-channel mean / biased variance of the bf16 output
    rows = hip.conv_tile_rows(K)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    M = yf.shape[0]
    assert st.shape == ((M + rows - 1) // rows, 2, K)
    mean = st[:, 0].sum(0) / M
    n = torch.tensor([min(rows, M - i * rows) for i in range(st.shape[0])], device="cuda", dtype=torch.float32)
    var = (st[:, 1].sum(0) + (n[:, None] * (st[:, 0] / n[:, None] - mean) ** 2).sum(0)) / M
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var, yf.var(0, unbiased=False), rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("N,C,H,K,R,stride", SHAPES)
def test_conv_dgrad(hip, N, C, H, K, R, stride):
    x, w = _mk(N, C, H, K, R, 2)
    pad = (R - 1) // 2
    xf = x.float().requires_grad_()
    ref = F.conv2d(xf, w.float(), stride=stride, padding=pad)
    g = torch.Generator(device="cuda").manual_seed(3)
    dy = torch.randn(ref.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    ref.backward(dy.float())
    wt = hip.conv_weight_t(w)
    assert wt.shape == (C, R * R * K)
    dx = hip.conv_dgrad(dy, wt, C, R, R, H, H, stride, pad)
    assert dx.shape == x.shape and dx.is_contiguous(memory_format=torch.channels_last)
    assert _rel(dx, xf.grad) < 1e-2
    # a joining branch gradient summed in the epilogue (1×1 stride 2: the untouched
    # parity classes take the addend as is)
    add = torch.randn(x.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    dxa = hip.conv_dgrad(dy, wt, C, R, R, H, H, stride, pad, add)
    assert _rel(dxa, xf.grad + add.float()) < 1e-2


@pytest.mark.parametrize("T,N,K", [(1024, 256, 512), (2048, 512, 128), (512, 256, 64)])
def test_gemm_nt_add(hip, T, N, K):
    """c = a·bᵀ + r on both mainloops (K ≥ 256: the 4-wave kernel; K = 64 / 128: the 8-wave one)."""
    g = torch.Generator(device="cuda").manual_seed(T + K)
    a = torch.randn(T, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    r = torch.randn(T, N, device="cuda", generator=g).bfloat16()
    c = hip.gemm_nt_add(a, b, r)
    assert _rel(c, a.float() @ b.float().t() + r.float()) < 1e-2


def test_bn_from_tile_stats_matches_stats_pass(hip):
    """BatchNorm forward from the conv epilogue's tile partials equals the
    stats-pass BatchNorm (bn_act_fwd) on the same activation."""
    x, w = _mk(4, 64, 14, 64, 3, 5)
    y, st = hip.conv_fwd(x, w, 1, 1, True)
    g = torch.Generator(device="cuda").manual_seed(6)
    gamma = torch.rand(64, device="cuda", generator=g) + 0.5
    beta = torch.randn(64, device="cuda", generator=g) * 0.1
    rm1, rv1 = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
    rm2, rv2 = rm1.clone(), rv1.clone()
    a, m_a, i_a, _ = hip.bn_act_fwd(y, None, gamma, beta, rm1, rv1, 1e-5, 0.1, True)
    b, m_b, i_b, _ = hip.bn_act_fwd_tiles(y, st, hip.conv_tile_rows(64), None, gamma, beta, rm2, rv2, 1e-5, 0.1, True)
    torch.testing.assert_close(m_b, m_a, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(i_b, i_a, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rv2, rv1, rtol=1e-3, atol=1e-5)
    assert _rel(b, a) < 1e-2


@pytest.mark.parametrize("N,C,H,K,R,stride", SHAPES)
def test_conv_wgrad(hip, N, C, H, K, R, stride):
    """Weight gradient (split-K over tokens, fp32 partials folded in order) vs
    fp32 autograd, into a fresh tensor and accumulated into an existing one."""
    x, w = _mk(N, C, H, K, R, 4)
    pad = (R - 1) // 2
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=stride, padding=pad)
    g = torch.Generator(device="cuda").manual_seed(8)
    dy = torch.randn(ref.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    ref.backward(dy.float())
    dw = hip.conv_wgrad(dy, x, R, R, stride, pad)
    assert dw.shape == w.shape and dw.dtype == torch.float32
    assert _rel(dw, wf.grad) < 5e-3
    base = torch.randn_like(dw).contiguous(memory_format=torch.channels_last)
    acc = base.clone()
    hip.conv_wgrad(dy, x, R, R, stride, pad, out=acc)
    assert _rel(acc - base, wf.grad) < 5e-3


def test_bottleneck_hip_conv_path_matches_framework_conv():
    """A ResNet-50 downsampling bottleneck (3×3 stride 2 + strided 1×1 on the HIP
    implicit GEMM, BN statistics from its epilogue) against the same block on
    the framework's convolutions: output, input gradient and every parameter
    gradient agree to bf16 accuracy."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import Bottleneck

    torch.manual_seed(0)
    ds = torch.nn.Sequential(torch.nn.Conv2d(256, 512, 1, stride=2, bias=False), torch.nn.BatchNorm2d(512))
    a = Bottleneck(256, 128, stride=2, downsample=ds).cuda().to(memory_format=torch.channels_last)
    for mod in a.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    b = copy.deepcopy(a)
    x = torch.randn(4, 256, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for mod, hip_conv in ((a, True), (b, False)):
        prev = ops._HIP_CONV[0]
        ops._HIP_CONV[0] = hip_conv
        try:
            xx = x.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xx)
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._HIP_CONV[0] = prev
        outs.append((y, xx.grad))
    assert _rel(outs[0][0], outs[1][0]) < 2e-2
    assert _rel(outs[0][1], outs[1][1]) < 3e-2
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert _rel(pa.grad, pb.grad) < 3e-2, n


def test_layer4_bottleneck_ragged_tokens_matches_framework_conv():
    """A layer4 identity bottleneck (2048 → 512 → 2048 channels, 7×7) at 3
    images: 147 tokens, not a multiple of gemm_dw's 64-token k-tile, so its 1×1
    weight gradients must leave the token-major GEMM for the implicit-GEMM
    weight gradient (the GEMM's False return was once ignored and an unwritten
    buffer used as the gradient).  Every parameter gradient against the
    framework's convolutions."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import Bottleneck

    torch.manual_seed(0)
    a = Bottleneck(2048, 512).cuda().to(memory_format=torch.channels_last)
    for mod in a.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    b = copy.deepcopy(a)
    x = torch.randn(3, 2048, 7, 7, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    grads = []
    for mod, hip_conv in ((a, True), (b, False)):
        prev = ops._HIP_CONV[0]
        ops._HIP_CONV[0] = hip_conv
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(x)
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._HIP_CONV[0] = prev
        grads.append({n: q.grad.clone() for n, q in mod.named_parameters()})
    for n in grads[1]:
        assert torch.isfinite(grads[0][n]).all(), n
        assert _rel(grads[0][n], grads[1][n]) < 3e-2, n


@pytest.mark.parametrize("N,C,H,K,stride", [(2, 64, 16, 64, 1), (3, 128, 7, 128, 2), (2, 128, 16, 128, 2)])
def test_conv_dgrad_bn_partials(hip, N, C, H, K, stride):
    """The input gradient's epilogue BatchNorm partials, folded by
    bn_act_bwd_part, give the same dx / dgamma / dbeta as the stats-pass
    BatchNorm backward on the same (dy, x)."""
    g = torch.Generator(device="cuda").manual_seed(11)
    bx = torch.randn(N, C, H, H, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    gamma = torch.rand(C, device="cuda", generator=g) + 0.5
    beta = torch.randn(C, device="cuda", generator=g) * 0.2
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y, mean, invstd, _ = hip.bn_act_fwd(bx, None, gamma, beta, rm, rv, 1e-5, 0.1, True)
    w = (torch.randn(K, C, 3, 3, device="cuda", generator=g) / (9 * C) ** 0.5).bfloat16()
    w = w.contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 - 3) // stride + 1
    dy = torch.randn(N, K, Ho, Ho, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    wt = hip.conv_weight_t(w)
    dx_plain = hip.conv_dgrad(dy, wt, C, 3, 3, H, H, stride, 1)
    dx, part = hip.conv_dgrad_bn(dy, wt, 3, 3, stride, 1, bx, mean, invstd, gamma, beta, True)
    assert torch.equal(dx, dx_plain)
    a = hip.bn_act_bwd(dx, None, bx, mean, invstd, gamma, beta, True, False, None, None)
    b = hip.bn_act_bwd_part(part, dx, None, bx, mean, invstd, gamma, beta, True, False, None, None)
    for u, v in ((a[0], b[0]), (a[2], b[2]), (a[3], b[3])):
        assert _rel(v, u) < 2e-3


def test_bottleneck_bn_link_matches_unlinked():
    """ResNet bottleneck with bn1's backward statistics from conv2's input-gradient
    epilogue (ops._BNLink) vs the stats-pass backward: same gradients, and the
    link was actually taken."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import Bottleneck

    torch.manual_seed(1)
    a = Bottleneck(256, 64).cuda().to(memory_format=torch.channels_last)
    for mod in a.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    b = copy.deepcopy(a)
    x = torch.randn(4, 256, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for mod, link in ((a, True), (b, False)):
        prev, used = ops._BN_LINK[0], ops._BN_LINK_USED[0]
        ops._BN_LINK[0] = link
        try:
            xx = x.clone().requires_grad_()
            y = mod(xx)
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._BN_LINK[0] = prev
        # bn1 → conv2 and bn2 → conv3 (both implicit-GEMM input gradients)
        assert (ops._BN_LINK_USED[0] - used) == (2 if link else 0)
        outs.append(xx.grad)
    assert _rel(outs[0], outs[1]) < 1e-2
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert _rel(pa.grad, pb.grad) < 1e-2, n


@pytest.mark.parametrize("N,C,H,K,R,stride", [(4, 256, 16, 256, 3, 1), (8, 256, 16, 512, 3, 2), (4, 512, 8, 512, 3, 1),
                                              (8, 256, 16, 128, 1, 1), (16, 256, 8, 512, 1, 2), (4, 1024, 8, 256, 1, 1),
                                              (8, 128, 16, 128, 3, 1), (8, 128, 16, 512, 1, 1)])
def test_conv_wgrad_dw4_gathered(hip, N, C, H, K, R, stride):
    """The weight gradient on gemm_dw4's 256 × 256 mainloop with the activation
    gathered per tap (zero padding through out-of-range buffer offsets; Kout = 128:
    half-height tiles; R·S·C = 1152 / 128: a zero-padded last 256-column tile)
    against fp32 autograd and against the 128 × 128 kernel."""
    x, w = _mk(N, C, H, K, R, 9)
    pad = (R - 1) // 2
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=stride, padding=pad)
    g = torch.Generator(device="cuda").manual_seed(10)
    dy = torch.randn(ref.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    ref.backward(dy.float())
    assert (dy.numel() // K) % 128 == 0  # the shapes take the gathered path
    prev = hip.conv_wgrad_mode(1)
    try:
        dw4 = hip.conv_wgrad(dy, x, R, R, stride, pad)
        hip.conv_wgrad_mode(0)
        dw1 = hip.conv_wgrad(dy, x, R, R, stride, pad)
    finally:
        hip.conv_wgrad_mode(prev)
    assert dw4.shape == w.shape and dw4.dtype == torch.float32
    assert _rel(dw4, wf.grad) < 5e-3
    assert _rel(dw4, dw1) < 1e-4


def test_bn_residual_relu_mask_matches_saved_output(hip):
    """BatchNorm + residual + ReLU: the backward from the forward's 1-bit ReLU mask
    equals the backward from the saved bf16 output, bit for bit."""
    g = torch.Generator(device="cuda").manual_seed(12)
    x = torch.randn(4, 256, 14, 14, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    res = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
    gamma = torch.rand(256, device="cuda", generator=g) + 0.5
    beta = torch.randn(256, device="cuda", generator=g) * 0.2
    y, mean, invstd, mask = hip.bn_act_fwd(x, res, gamma, beta, None, None, 1e-5, 0.1, True)
    assert mask.dtype == torch.uint8 and mask.numel() == x.numel() // 8
    yl = y.permute(0, 2, 3, 1).reshape(-1)
    bits = ((mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).reshape(-1)
    assert torch.equal(bits.bool(), yl.float() > 0)
    dy = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
    a = hip.bn_act_bwd(dy, y, x, mean, invstd, gamma, beta, True, True, None, None)
    b = hip.bn_act_bwd(dy, mask, x, mean, invstd, gamma, beta, True, True, None, None)
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("N,C,H,stride", [(8, 64, 16, 1), (3, 64, 7, 1), (16, 64, 28, 1), (8, 128, 16, 1),
                                           (3, 128, 7, 1), (8, 128, 16, 2), (4, 64, 14, 2)])
def test_conv_wgrad_tap_groups(hip, N, C, H, stride):
    """The tap-group 3×3 weight gradient (C = Kout = 64: all nine taps per
    workgroup; 128: one kernel row of three) — dY staged once per k-step for the
    group's gathered X tiles — against fp32 autograd and the per-tap / dw4
    kernels; token counts with a partial last k-step (3 × 7 × 7), stride 2."""
    x, w = _mk(N, C, H, C, 3, 13)
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=stride, padding=1)
    g = torch.Generator(device="cuda").manual_seed(14)
    dy = torch.randn(ref.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    ref.backward(dy.float())
    prev = hip.conv_wgrad_c64_mode(1)
    try:
        dw = hip.conv_wgrad(dy, x, 3, 3, stride, 1)
        hip.conv_wgrad_c64_mode(0)
        dw1 = hip.conv_wgrad(dy, x, 3, 3, stride, 1)
    finally:
        hip.conv_wgrad_c64_mode(prev)
    assert _rel(dw, wf.grad) < 5e-3
    assert _rel(dw, dw1) < 1e-4


@pytest.mark.parametrize("N,H,W", [(2, 224, 224), (3, 30, 30), (2, 64, 48), (1, 8, 14)])
def test_stem_space_to_depth(hip, N, H, W):
    """The 7×7 / stride-2 / pad-3 stem as a 4×4 stride-1 convolution over the
    16-channel space-to-depth image: output and BatchNorm tile statistics vs
    fp32 F.conv2d, weight gradient (fresh and accumulated) vs fp32 autograd;
    token counts with a partial last tile / k-step (3 × 15 × 15, 1 × 4 × 7)."""
    g = torch.Generator(device="cuda").manual_seed(H + W)
    x = torch.randn(N, 3, H, W, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) / 147 ** 0.5).bfloat16()
    w = w.contiguous(memory_format=torch.channels_last)
    assert hip.stem_ok(N, H, W, 3, 64)
    y, st, z = hip.stem_fwd(x, w, True)
    wf = w.float().requires_grad_()
    ref = F.conv2d(x.float(), wf, stride=2, padding=3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert z.shape == (N, 16, H // 2, W // 2)
    assert _rel(y, ref) < 1e-2
    rows = hip.stem_tile_rows()
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
    M = yf.shape[0]
    assert st.shape == ((M + rows - 1) // rows, 2, 64)
    mean = st[:, 0].sum(0) / M
    n = torch.tensor([min(rows, M - i * rows) for i in range(st.shape[0])], device="cuda", dtype=torch.float32)
    var = (st[:, 1].sum(0) + (n[:, None] * (st[:, 0] / n[:, None] - mean) ** 2).sum(0)) / M
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(var, yf.var(0, unbiased=False), rtol=1e-3, atol=1e-5)
    dy = torch.randn(ref.shape, device="cuda", generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    ref.backward(dy.float())
    dw = hip.stem_wgrad(dy, z)
    assert dw.shape == w.shape and dw.dtype == torch.float32
    assert _rel(dw, wf.grad) < 5e-3
    base = torch.randn_like(dw).contiguous(memory_format=torch.channels_last)
    acc = base.clone()
    hip.stem_wgrad(dy, z, acc)
    assert _rel(acc - base, wf.grad) < 5e-3


def test_resnet_stem_hip_path_matches_framework_conv():
    """ResNet-50's stem block (conv1 → bn1 → ReLU → max-pool) on the
    space-to-depth kernels and on the framework convolution (both bf16), each
    against the same block in fp32: the HIP path's output and conv / BatchNorm
    parameter gradients are as close to fp32 as the framework's (the conv
    weight gradient sums a BatchNorm-centred dY over every pixel, so both bf16
    paths sit a few % off fp32 there)."""
    import copy

    from paddle_operator_amd import ops

    torch.manual_seed(0)
    a = torch.nn.ModuleDict({"conv1": torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False),
                             "bn1": torch.nn.BatchNorm2d(64)}).cuda().to(memory_format=torch.channels_last)
    torch.nn.init.uniform_(a["bn1"].weight, 0.5, 1.5)
    b, c = copy.deepcopy(a), copy.deepcopy(a)
    x = torch.randn(4, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for mod, hip_conv, xin in ((a, True, x), (b, False, x), (c, False, x.float())):
        prev = ops._HIP_CONV[0]
        ops._HIP_CONV[0] = hip_conv
        try:
            assert ops._stem_ok(mod["conv1"], xin) == hip_conv
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=xin.dtype == torch.bfloat16):
                y = ops.max_pool_3x3s2(ops.conv_bn_act(mod["conv1"], mod["bn1"], xin))
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._HIP_CONV[0] = prev
        outs.append(y)
    assert _rel(outs[0], outs[2]) < 2e-2 and _rel(outs[1], outs[2]) < 2e-2
    for (n, pa), (_, pb), (_, pc) in zip(a.named_parameters(), b.named_parameters(), c.named_parameters()):
        e_hip, e_fw = _rel(pa.grad, pc.grad), _rel(pb.grad, pc.grad)
        assert e_hip < 1.5 * e_fw + 1e-2, (n, e_hip, e_fw)
    torch.testing.assert_close(a["bn1"].running_mean, c["bn1"].running_mean, rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("N,H", [(4, 64), (3, 30), (2, 18)])
def test_stem_bn_relu_pool_fused_matches_unfused(N, H):
    """The stem's BatchNorm + ReLU + 3×3/2 max-pool in one pass each way
    (ops._BNReluPoolFn) against the same block through bn_act + max-pool: the
    pooled output bit-identical, the conv / BatchNorm gradients and running
    statistics equal to bf16 accuracy (odd pooled sizes: 15 → 8, 9 → 5)."""
    import copy

    from paddle_operator_amd import ops

    torch.manual_seed(N + H)
    a = torch.nn.ModuleDict({"conv1": torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False),
                             "bn1": torch.nn.BatchNorm2d(64)}).cuda().to(memory_format=torch.channels_last)
    torch.nn.init.uniform_(a["bn1"].weight, -0.5, 1.5)  # some negative scales: the max is not at max(x)
    torch.nn.init.uniform_(a["bn1"].bias, -0.2, 0.2)
    b = copy.deepcopy(a)
    x = torch.randn(N, 3, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for mod, fused in ((a, True), (b, False)):
        prev = ops._STEM_POOL[0]
        ops._STEM_POOL[0] = fused
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = ops.conv_bn_relu_maxpool(mod["conv1"], mod["bn1"], x)
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._STEM_POOL[0] = prev
        outs.append(y)
    assert outs[0].shape == outs[1].shape == (N, 64, (H // 2 - 1) // 2 + 1, (H // 2 - 1) // 2 + 1)
    assert torch.equal(outs[0], outs[1])
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert _rel(pa.grad, pb.grad) < 1e-2, n
    torch.testing.assert_close(a["bn1"].running_mean, b["bn1"].running_mean)
    torch.testing.assert_close(a["bn1"].running_var, b["bn1"].running_var)


def test_stem_arena_grads_match_autograd():
    """The stem's weight gradient (stem_wgrad, accumulated into the fp32 arena
    slice) and its BatchNorm γ/β gradients (pool_bn_bwd into the arena) on the
    arena-direct path equal the same kernels' returned gradients under plain
    autograd — a dropped, doubled or misplaced arena write is an O(1) error."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.parallel.flat import FlatParams

    torch.manual_seed(3)
    a = torch.nn.ModuleDict({"conv1": torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False),
                             "bn1": torch.nn.BatchNorm2d(64)}).cuda().to(memory_format=torch.channels_last)
    torch.nn.init.uniform_(a["bn1"].weight, 0.5, 1.5)
    b = copy.deepcopy(a)
    flat = FlatParams(a, dtype=torch.float32, device="cuda")
    x = torch.randn(4, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    flat.zero_grad()
    for mod in (a, b):
        assert ops._stem_ok(mod["conv1"], x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = ops.conv_bn_relu_maxpool(mod["conv1"], mod["bn1"], x)
        (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
    torch.cuda.synchronize()
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert pa.grad.data_ptr() >= flat.grads.data_ptr(), n
        assert _rel(pa.grad, pb.grad) < 2e-3, n


@pytest.mark.parametrize("downsample", [False, True])
def test_identity_bottleneck_residual_mask_in_dx_epilogue(downsample):
    """bn3's residual gradient dy ⊙ relu' is not written by its BatchNorm
    backward: in an identity bottleneck conv1's dX GEMM epilogue forms it
    (gemm_nt_add EPI 6), in a downsample bottleneck the downsample BatchNorm's
    backward applies the mask (bitmask mode) — same output and gradients as with
    the hand-off off (PDO_RES_MASK=0 path), and the hand-off is taken."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import Bottleneck

    torch.manual_seed(5)
    ds = (torch.nn.Sequential(torch.nn.Conv2d(256, 512, 1, stride=2, bias=False), torch.nn.BatchNorm2d(512))
          if downsample else None)
    a = Bottleneck(256, 128 if downsample else 64, stride=2 if downsample else 1,
                   downsample=ds).cuda().to(memory_format=torch.channels_last)
    for mod in a.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    b = copy.deepcopy(a)
    x = torch.randn(4, 256, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for mod, on in ((a, True), (b, False)):
        prev = ops._RES_MASK[0], ops._DS_FUSED[0]
        # (the downsample case exercises the two-pass tail's hand-off: the fused
        # tail, _BNActBNResFn, needs none — test_downsample_block_bn_pair_in_one_apply)
        ops._RES_MASK[0], ops._DS_FUSED[0] = on, False
        used = ops._RES_MASK_USED[0]
        try:
            xx = x.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xx)
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._RES_MASK[0], ops._DS_FUSED[0] = prev
        assert (ops._RES_MASK_USED[0] - used) == (1 if on else 0)
        outs.append((y, xx.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert _rel(outs[0][1], outs[1][1]) < 1e-2
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert _rel(pa.grad, pb.grad) < 1e-2, n


@pytest.mark.parametrize("T,N,K", [(4096, 1024, 1024), (2048, 256, 64)])
def test_gemm_nt_add_masked(hip, T, N, K):
    """c = a·bᵀ + r ⊙ keep (gemm_nt EPI 6) on the 4-wave (K ≥ 256) and 8-wave
    (K = 64) mainloops against fp32."""
    g = torch.Generator(device="cuda").manual_seed(T + N + K)
    a = torch.randn(T, K, device="cuda", generator=g).bfloat16()
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    r = torch.randn(T, N, device="cuda", generator=g).bfloat16()
    mask = torch.randint(0, 256, (T * N // 8,), device="cuda", generator=g, dtype=torch.int64).to(torch.uint8)
    keep = ((mask.view(-1, 1) >> torch.arange(8, device="cuda", dtype=torch.uint8)) & 1).view(T, N).float()
    c = hip.gemm_nt_add(a, b, r, mask=mask)
    assert _rel(c, a.float() @ b.float().t() + r.float() * keep) < 1e-2


def test_downsample_compact_input_gradient():
    """A stride-2 downsample bottleneck: the downsample's input gradient is
    computed compact and added into conv1's dX at the stride-2 pixels
    (ops._CompactGradLink, conv_stride2_add) — same input / parameter gradients
    as the zero-filled full-resolution path (PDO_DS_COMPACT=0), hand-off taken."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import Bottleneck

    torch.manual_seed(9)
    ds = torch.nn.Sequential(torch.nn.Conv2d(256, 512, 1, stride=2, bias=False), torch.nn.BatchNorm2d(512))
    a = Bottleneck(256, 128, stride=2, downsample=ds).cuda().to(memory_format=torch.channels_last)
    for mod in a.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    b = copy.deepcopy(a)
    x = torch.randn(4, 256, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for mod, on in ((a, True), (b, False)):
        prev = ops._DS_COMPACT[0]
        ops._DS_COMPACT[0] = on
        used = ops._DS_COMPACT_USED[0]
        try:
            xx = x.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xx)
            (y.float() * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
        finally:
            ops._DS_COMPACT[0] = prev
        assert (ops._DS_COMPACT_USED[0] - used) == (1 if on else 0)
        outs.append((y, xx.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert _rel(outs[0][1], outs[1][1]) < 1e-2
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert _rel(pa.grad, pb.grad) < 1e-2, n


@pytest.mark.parametrize("cin,width,stride,hw", [(256, 128, 2, 16), (64, 64, 1, 16), (1024, 512, 2, 14)])
def test_downsample_block_bn_pair_in_one_apply(cin, width, stride, hw):
    """A downsample bottleneck's tail ReLU(bn3(conv3) + bn_ds(conv_ds)) in one
    apply pass (ops._BNActBNResFn: the downsample BatchNorm's output never
    materialised) — same output, input / parameter gradients and running
    statistics as the two-pass path (PDO_DS_BN_FUSED=0); also against an fp32
    copy of the block on the framework ops."""
    import copy

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import Bottleneck

    torch.manual_seed(13)
    ds = torch.nn.Sequential(torch.nn.Conv2d(cin, width * 4, 1, stride=stride, bias=False),
                             torch.nn.BatchNorm2d(width * 4))
    a = Bottleneck(cin, width, stride=stride, downsample=ds).cuda().to(memory_format=torch.channels_last)
    for mod in a.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
            torch.nn.init.uniform_(mod.bias, -0.2, 0.2)
    b = copy.deepcopy(a)
    f = copy.deepcopy(a).float()
    x = torch.randn(4, cin, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    wgt = None
    outs = []
    for mod, on in ((a, True), (b, False)):
        prev = ops._DS_FUSED[0]
        ops._DS_FUSED[0] = on
        try:
            xx = x.clone().requires_grad_()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mod(xx)
            wgt = torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)
            (y.float() * wgt).sum().backward()
        finally:
            ops._DS_FUSED[0] = prev
        outs.append((y, xx.grad))
    # the residual enters the apply in fp32 instead of rounded to bf16 first: the
    # two paths differ by bf16 rounding, so each is held against an fp32 copy of
    # the block on the framework ops and the fused one may not be the worse
    assert _rel(outs[0][0], outs[1][0]) < 1e-2
    for (n, ba), (_, bb) in zip(a.named_buffers(), b.named_buffers()):
        if ba.dtype.is_floating_point:
            torch.testing.assert_close(ba, bb, rtol=1e-3, atol=1e-4, msg=n)
    prev = ops._HIP_CONV[0], ops._BN_FUSED[0]
    ops._HIP_CONV[0], ops._BN_FUSED[0] = False, False
    try:
        xf = x.float().requires_grad_()
        yf = f(xf)
        (yf * wgt).sum().backward()
    finally:
        ops._HIP_CONV[0], ops._BN_FUSED[0] = prev
    e_fused, e_two = _rel(outs[0][0].float(), yf), _rel(outs[1][0].float(), yf)
    assert e_fused < 3e-2 and e_fused <= 1.25 * e_two + 1e-3, (e_fused, e_two)
    e_fused, e_two = _rel(outs[0][1].float(), xf.grad), _rel(outs[1][1].float(), xf.grad)
    assert e_fused < 0.15 and e_fused <= 1.25 * e_two + 1e-3, ("dx", e_fused, e_two)
    for (n, pa), (_, pb), (_, pf) in zip(a.named_parameters(), b.named_parameters(), f.named_parameters()):
        e_fused, e_two = _rel(pa.grad.float(), pf.grad), _rel(pb.grad.float(), pf.grad)
        assert e_fused < 0.15 and e_fused <= 1.25 * e_two + 1e-3, (n, e_fused, e_two)


@pytest.mark.parametrize("N,C,HW", [(256, 2048, 7), (4, 64, 5)])
def test_global_avg_pool_channels_last_grad(N, C, HW):
    """ops.global_avg_pool (HIP backward: dy / HW written straight into a
    channels_last gradient) against the framework's adaptive_avg_pool2d in fp32."""
    from paddle_operator_amd import ops

    x = torch.randn(N, C, HW, HW, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_()
    y = ops.global_avg_pool(xa)
    dy = torch.randn(N, C, device="cuda").bfloat16()
    y.backward(dy)
    xr = x.float().requires_grad_()
    yr = torch.flatten(torch.nn.functional.adaptive_avg_pool2d(xr, 1), 1)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert xa.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xa.grad.float(), xr.grad, rtol=8e-3, atol=1e-6)
