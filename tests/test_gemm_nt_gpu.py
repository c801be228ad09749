"""gemm_nt (csrc/hip/gemm_nt.hip) numerics against plain PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from paddle_operator_amd import _native
    return _native.require_hip()


def _mk(M, N, K, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16, generator=g) * 0.1
    return x, w, b


def _gelu_grad(x):
    x = x.detach().requires_grad_(True)
    (g,) = torch.autograd.grad(F.gelu(x, approximate="tanh").sum(), x)
    return g


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (768, 256, 192), (512, 1024, 256), (2304, 512, 128)])
def test_plain_and_bias(hip, M, N, K):
    x, w, b = _mk(M, N, K)
    ref = x.float() @ w.float().t()
    c = hip.gemm_nt(x, w)
    torch.testing.assert_close(c.float(), ref, atol=2e-2, rtol=1e-2)
    cb = hip.gemm_nt(x, w, b)
    torch.testing.assert_close(cb.float(), ref + b.float(), atol=2e-2, rtol=1e-2)


def test_gelu_epilogue(hip):
    M, N, K = 1024, 512, 256
    x, w, b = _mk(M, N, K, 1)
    pre, y = hip.gemm_nt_gelu(x, w, b)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(pre.float(), ref, atol=2e-2, rtol=1e-2)
    # the activation is computed from the bf16-rounded pre-activation (as the unfused path)
    torch.testing.assert_close(y.float(), F.gelu(pre.float() + b.float(), approximate="tanh"), atol=1e-2, rtol=1e-2)
    # and the standalone HIP bias-GELU kernel on the same (bf16) input to a bf16
    # ulp: the row epilogue applies GELU to the fp32 pre-activation
    torch.testing.assert_close(y.float(), hip.bias_gelu_fwd(pre, b).float(), atol=1e-2, rtol=1e-2)


def test_dgelu_epilogue_and_bias_grad(hip):
    M, N, K = 1024, 512, 256
    x, w, b = _mk(M, N, K, 2)
    pre = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    dx, db = hip.gemm_nt_dgelu(x, w, pre, b)
    dy = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    ref = dy * _gelu_grad(pre.float() + b.float())
    torch.testing.assert_close(dx.float(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(db.float(), ref.sum(0), atol=0.5, rtol=2e-2)
    # accumulate into an existing (arena) gradient
    acc = torch.ones(N, device="cuda", dtype=torch.bfloat16)
    (dx2,) = hip.gemm_nt_dgelu(x, w, pre, b, db_out=acc)
    assert torch.equal(dx2, dx)
    torch.testing.assert_close(acc.float(), 1.0 + ref.sum(0), atol=0.5, rtol=2e-2)


def test_rejects_unsupported_shapes(hip):
    assert not hip.gemm_nt_supported(300, 256, 64)
    assert not hip.gemm_nt_supported(256, 256, 96)
    assert hip.gemm_nt_supported(65536, 4096, 1024)
    x, w, _ = _mk(320, 256, 64)
    with pytest.raises(RuntimeError):
        hip.gemm_nt(x, w)


# impls on the 4-wave mainloop (gemm_nt4.hip): its row epilogue takes GELU / GELU'
# on the fp32 product (impl 2: with the deferred store drain)
ROW_EPILOGUE_IMPLS = {1}


@pytest.mark.parametrize("M,N,K", [(512, 256, 256), (256, 768, 384), (1024, 512, 2048), (768, 256, 128)])
def test_nt4_mainloop_matches_ring(hip, M, N, K):
    """The 4-wave mainloop (gemm_nt4.hip, both store-drain forms) runs the k-tiles
    in the same order as the 8-wave ring: outputs equal bit for bit (the row
    epilogue's GELU / GELU' forms to a bf16 rounding step); K = 128
    falls back to the ring (the 4-wave loop needs ≥ 4 even k-tiles)."""
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    bias = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2, generator=g)
    prev = hip.gemm_nt_impl(0)
    try:
        ref = hip.gemm_nt(a, b, bias)
        ref_p, ref_y = hip.gemm_nt_gelu(a, b, bias)
        ref_dx, ref_db = hip.gemm_nt_dgelu(a, b, pre, bias)
        for impl in (1,):
            hip.gemm_nt_impl(impl)
            # the MFMAs take A as SrcA (row-major accumulators): the products and
            # their k order are the ring's, so they still match bitwise
            assert torch.equal(hip.gemm_nt(a, b, bias), ref), impl
            p, y = hip.gemm_nt_gelu(a, b, bias)
            dx, db = hip.gemm_nt_dgelu(a, b, pre, bias)
            assert torch.equal(p, ref_p), impl
            if impl in ROW_EPILOGUE_IMPLS:
                # the row epilogue takes GELU / GELU' on the fp32 product instead of
                # its bf16 rounding: equal to a bf16 rounding step
                torch.testing.assert_close(y.float(), ref_y.float(), atol=2e-2, rtol=1e-2)
                torch.testing.assert_close(dx.float(), ref_dx.float(), atol=2e-2, rtol=1e-2)
            else:
                assert torch.equal(y, ref_y) and torch.equal(dx, ref_dx), impl
            # bias-gradient partials are summed in another order: fp32 rounding only
            # (row epilogue: sums of the unrounded dX, so up to a bf16 step per row)
            atol = 2e-2 * ref_db.float().abs().max().item() if impl in ROW_EPILOGUE_IMPLS else 2e-2
            torch.testing.assert_close(db.float(), ref_db.float(), rtol=2e-2, atol=atol)
        exact = a.float() @ b.float().t() + bias.float()
        torch.testing.assert_close(ref.float(), exact, rtol=2e-2, atol=6e-2)
    finally:
        hip.gemm_nt_impl(prev)


@pytest.mark.parametrize("M,N,K,impl", [(65536, 4096, 1024, 1), (3328, 1024, 3072, 1), (65536, 1024, 4096, 1),
                                        (3328, 50304, 1024, 1), (2048, 768, 1024, 1)])
def test_nt4_production_shapes_vs_fp32(hip, M, N, K, impl):
    """Production-size grids: M = 65536 (4096 tiles: XCD remap over every tile,
    grouped order across 32 groups of 8 tile rows) and M = 3328 (13 tile rows,
    tiles_m % 8 != 0: the last group is short), full output against fp32."""
    g = torch.Generator(device="cuda").manual_seed(11)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
    bias = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-0.1, 0.1, generator=g)
    prev = hip.gemm_nt_impl(impl)
    try:
        c = hip.gemm_nt(a, b, bias)
    finally:
        hip.gemm_nt_impl(prev)
    ref = torch.addmm(bias.float(), a.float(), b.float().t())
    err = (c.float() - ref).abs()
    tol = 1e-2 + 8e-3 * ref.abs()
    assert bool((err <= tol).all()), f"max err {err.max().item():.4f} at {int(err.argmax())}"


@pytest.mark.parametrize("impl", [1])
def test_nt4_half_width_last_tile(hip, impl):
    """N % 256 = 128 (the 50304-column LM head) on the row-accumulator variants:
    the last tile column is half wide; its upper-half waves store nothing and
    their B reads stay in bounds.  Plain, bias, GELU and dGELU epilogues vs fp32."""
    M, N, K = 768, 640, 512
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-0.1, 0.1, generator=g)
    bias = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-0.1, 0.1, generator=g)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2, generator=g)
    prev = hip.gemm_nt_impl(impl)
    try:
        assert hip.gemm_nt_supported(M, N, K)
        c = hip.gemm_nt(a, b, None)
        cb = hip.gemm_nt(a, b, bias)
        p, y = hip.gemm_nt_gelu(a, b, bias)
        dx, db = hip.gemm_nt_dgelu(a, b, pre, bias)
    finally:
        hip.gemm_nt_impl(prev)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(c.float(), ref, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(cb.float(), ref + bias.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(p.float(), ref, rtol=1e-2, atol=1e-2)
    x = p.float() + bias.float()
    torch.testing.assert_close(y.float(), torch.nn.functional.gelu(x, approximate="tanh"), rtol=2e-2, atol=2e-2)
    xp = (pre.float() + bias.float()).requires_grad_(True)
    torch.nn.functional.gelu(xp, approximate="tanh").backward(ref.to(torch.bfloat16).float())
    torch.testing.assert_close(dx.float(), xp.grad, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(db.float(), xp.grad.sum(0), rtol=3e-2, atol=0.5)


@pytest.mark.parametrize("M,N", [(16384, 4096), (2048, 1024), (65536, 4096), (4352, 2048)])
@pytest.mark.parametrize("impl", [1])
def test_nt4_fused_epilogues_many_tiles_vs_fp32(hip, impl, M, N):
    """The GELU and GELU'+bias-grad epilogues against fp32 (pre-activation,
    activation, input gradient, bias gradient) at K = 1024 on persistent grids
    with 4 tiles per workgroup (16384 x 4096), one (2048 x 1024), 16 (the
    GPT-2-medium fc1 / fc2-dX shape) and an uneven 2-3 (4352 x 2048: 136 tiles,
    17 tile rows)."""
    K = 1024
    g = torch.Generator(device="cuda").manual_seed(21)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
    bias = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-0.1, 0.1, generator=g)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-2, 2, generator=g)
    prev = hip.gemm_nt_impl(impl)
    try:
        p, y = hip.gemm_nt_gelu(a, b, bias)
        dx, db = hip.gemm_nt_dgelu(a, b, pre, bias)
    finally:
        hip.gemm_nt_impl(prev)
    ref = a.float() @ b.float().t()
    tol = 1e-2 + 8e-3 * ref.abs()
    assert bool(((p.float() - ref).abs() <= tol).all())
    gl = torch.nn.functional.gelu(p.float() + bias.float(), approximate="tanh")
    assert bool(((y.float() - gl).abs() <= 1e-2 + 8e-3 * gl.abs()).all())
    xp = (pre.float() + bias.float()).requires_grad_(True)
    torch.nn.functional.gelu(xp, approximate="tanh").backward(ref.to(torch.bfloat16).float())
    assert bool(((dx.float() - xp.grad).abs() <= 2e-2 + 1e-2 * xp.grad.abs()).all())
    # the reference takes dy = bf16(A·Bᵀ), the epilogue the fp32 product:
    # per-row differences of 2^-9 |dy| add up like √M over the column
    torch.testing.assert_close(db.float(), xp.grad.sum(0), rtol=2e-2, atol=0.5 * (M / 16384) ** 0.5)



@pytest.mark.parametrize("M,N,K", [(65536, 4096, 1024), (4352, 2048, 1024), (768, 640, 512)])
def test_nt4_saved_gelu_grad_pair_vs_fp32(hip, M, N, K):
    """EPI 7 / 8: fc1 stores gelu'(x) (x = A·Bᵀ + bias in fp32) next to gelu(x);
    fc2's input gradient multiplies its fp32 product by the saved bf16 gelu' and
    sums the bias gradient.  Against fp32 (autograd of F.gelu on the exact
    pre-activation), at the GPT-2-medium shape, an uneven persistent grid and a
    half-width last tile column."""
    g = torch.Generator(device="cuda").manual_seed(31)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    w1 = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
    b1 = torch.empty(N, device="cuda", dtype=torch.bfloat16).uniform_(-0.1, 0.1, generator=g)
    dy = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    w2t = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
    gd, y = hip.gemm_nt_gelu(a, w1, b1, saved_grad=True)
    x = (a.float() @ w1.float().t() + b1.float()).requires_grad_(True)
    gl = F.gelu(x, approximate="tanh")
    (gref,) = torch.autograd.grad(gl.sum(), x)
    assert bool(((y.float() - gl).abs() <= 1e-2 + 8e-3 * gl.abs()).all())
    assert bool(((gd.float() - gref).abs() <= 1e-2 + 8e-3 * gref.abs()).all())
    dx, db = hip.gemm_nt_dgelu(dy, w2t, gd, b1, saved_grad=True)
    ref = (dy.float() @ w2t.float().t()) * gref
    assert bool(((dx.float() - ref).abs() <= 2e-2 + 1.6e-2 * ref.abs()).all())
    torch.testing.assert_close(db.float(), ref.sum(0), rtol=2e-2, atol=0.5 * (M / 16384) ** 0.5)
    acc = torch.ones(N, device="cuda", dtype=torch.bfloat16)
    (dx2,) = hip.gemm_nt_dgelu(dy, w2t, gd, b1, db_out=acc, saved_grad=True)
    assert torch.equal(dx2, dx)
    torch.testing.assert_close(acc.float(), 1.0 + ref.sum(0), rtol=2e-2, atol=0.5 * (M / 16384) ** 0.5 + 0.01)


@pytest.mark.parametrize("M,N,K", [(12544, 1024, 256), (50176, 256, 1024), (3328, 2048, 512), (768, 640, 512),
                                   (802816 // 4, 256, 64), (12544, 512, 128)])
def test_nt_bn_stats_epilogue_vs_fp32(hip, M, N, K):
    """EPI 9 (gemm_nt_stats): C = A·Bᵀ plus BatchNorm partials (Σ, Σ(x − x̄)²)
    of the bf16 outputs per row group — on the 4-wave mainloop a (256-row tile,
    wm) half: rows 256·tile + 128·wm + …, 128 rows; on the 8-wave ring (K < 256)
    the whole 256-row tile.  Checked per group against fp32 sums of the
    kernel's own bf16 output, and the merged column mean / variance against the
    fp32 product (ResNet-50 1×1 shapes, a half-width last tile column)."""
    g = torch.Generator(device="cuda").manual_seed(41)
    a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)
    b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-0.05, 0.05, generator=g)
    a[:, 0] = 8.0  # a column offset: |mean| ≫ std in some channels
    rows = hip.gemm_nt_stats_rows(K)
    assert rows == (128 if K >= 256 else 256)
    c, part = hip.gemm_nt_stats(a, b)
    ref = a.float() @ b.float().t()
    assert bool(((c.float() - ref).abs() <= 1e-2 + 8e-3 * ref.abs()).all())
    assert part.shape == (M // rows, 2, N)
    yg = c.float().view(M // rows, rows, N)
    s_ref = yg.sum(1)
    m2_ref = ((yg - yg.mean(1, keepdim=True)) ** 2).sum(1)
    torch.testing.assert_close(part[:, 0], s_ref, rtol=1e-4, atol=2e-3)
    torch.testing.assert_close(part[:, 1], m2_ref, rtol=2e-3, atol=2e-3)
    mean = part[:, 0].sum(0) / M
    var = (part[:, 1].sum(0) + (rows * (part[:, 0] / rows - mean) ** 2).sum(0)) / M
    torch.testing.assert_close(mean, ref.mean(0), rtol=1e-2, atol=2e-3)
    torch.testing.assert_close(var, ref.var(0, unbiased=False), rtol=2e-2, atol=1e-4)


@pytest.mark.parametrize("M,N,K", [(65536, 1024, 1024), (65536, 1024, 256), (3328, 50304, 512),
                                   (2048, 768, 4096)])
def test_nt4_dynamic_tile_order_matches_static(hip, M, N, K):
    """The dynamic per-XCD tile order (gemm_nt4_dynamic(1), an experiment switch) writes
    exactly what the static order does — every tile once, the same tile math —
    across more launches than the counter ring holds (each launch's last
    workgroup must leave its slot zeroed: a stale counter would skip tiles), with
    the fused epilogues, on a half-width last tile column and at nk = 4."""
    x, w, b = _mk(M, N, K, seed=7)
    y = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    prev = hip.gemm_nt4_dynamic(0)
    try:
        ref = (hip.gemm_nt(x, w), hip.gemm_nt(x, w, b), hip.gemm_nt_add(x, w, y))
        hip.gemm_nt4_dynamic(1)
        for it in range(300):  # > 256 slots: every slot reused
            got = hip.gemm_nt(x, w)
            if it % 50 == 0 or it == 299:
                assert torch.equal(got, ref[0]), it
        assert torch.equal(hip.gemm_nt(x, w, b), ref[1])
        assert torch.equal(hip.gemm_nt_add(x, w, y), ref[2])
    finally:
        hip.gemm_nt4_dynamic(prev)


def test_nt4_dynamic_tile_order_in_graph_replays(hip):
    """A dynamic-order launch captured in a HIP graph keeps its counter slot;
    every replay must find it zeroed again and cover all tiles."""
    x, w, _ = _mk(65536, 1024, 1024, seed=3)
    ref = hip.gemm_nt(x, w)
    prev = hip.gemm_nt4_dynamic(1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        out = hip.gemm_nt(x, w)
    torch.cuda.current_stream().wait_stream(s)
    try:
        for _ in range(5):
            out.zero_()
            g.replay()
            torch.cuda.synchronize()
            assert torch.equal(out, ref)
    finally:
        hip.gemm_nt4_dynamic(prev)
