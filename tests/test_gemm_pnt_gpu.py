"""gemm_pnt (csrc/hip/gemm_pnt.hip, persistent) numerics against plain PyTorch fp32
references, and bit-identity with gemm_nt.hip where the arithmetic is the same.

Shapes cover: tiles that do not divide the grid, workgroups with 1 tile, grids
smaller than the tile count (several tiles per workgroup, so the DMA ring and
the epilogue cross tile boundaries), and the minimum K (4 k-stages)."""
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


SHAPES = [(256, 256, 128, 0), (768, 512, 192, 0), (2048, 1024, 256, 3), (1280, 768, 1024, 5), (4096, 3072, 1024, 0)]


@pytest.mark.parametrize("M,N,K,grid", SHAPES)
def test_plain_and_bias(hip, M, N, K, grid):
    x, w, b = _mk(M, N, K)
    ref = x.float() @ w.float().t()
    (c,) = hip.gemm_pnt(x, w, 0, grid=grid)
    torch.testing.assert_close(c.float(), ref, atol=2e-2, rtol=1e-2)
    (cb,) = hip.gemm_pnt(x, w, 1, bias=b, grid=grid)
    torch.testing.assert_close(cb.float(), ref + b.float(), atol=2e-2, rtol=1e-2)
    if K % 64 == 0:  # same k-order MFMA chain as gemm_nt: identical bits
        assert torch.equal(c, hip.gemm_nt(x, w))


@pytest.mark.parametrize("grid", [0, 7])
def test_gelu_epilogue(hip, grid):
    M, N, K = 2048, 1024, 256
    x, w, b = _mk(M, N, K, 1)
    pre, y = hip.gemm_pnt(x, w, 2, bias=b, grid=grid)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(pre.float(), ref, atol=2e-2, rtol=1e-2)
    assert torch.equal(y, hip.bias_gelu_fwd(pre, b))
    p2, y2 = hip.gemm_nt_gelu(x, w, b)
    assert torch.equal(pre, p2) and torch.equal(y, y2)


@pytest.mark.parametrize("grid", [0, 5])
def test_dgelu_epilogue_and_bias_grad(hip, grid):
    M, N, K = 2048, 1024, 256
    x, w, b = _mk(M, N, K, 2)
    pre = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    dx, db = hip.gemm_pnt(x, w, 3, bias=b, pre=pre, grid=grid)
    dy = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    ref = dy * _gelu_grad(pre.float() + b.float())
    torch.testing.assert_close(dx.float(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(db.float(), dx.float().sum(0), atol=0.5, rtol=2e-2)
    dxn, _ = hip.gemm_nt_dgelu(x, w, pre, b)
    assert torch.equal(dx, dxn)
    acc = torch.ones(N, device="cuda", dtype=torch.bfloat16)
    (dx2,) = hip.gemm_pnt(x, w, 3, bias=b, pre=pre, db_out=acc, grid=grid)
    assert torch.equal(dx2, dx)
    torch.testing.assert_close(acc.float(), 1.0 + dx.float().sum(0), atol=0.5, rtol=2e-2)


def test_rejects_unsupported_shapes(hip):
    assert not hip.gemm_pnt_supported(300, 256, 128)
    assert not hip.gemm_pnt_supported(256, 256, 96)   # fewer than 4 k-stages
    assert not hip.gemm_pnt_supported(256, 256, 100)  # K % 32
    assert hip.gemm_pnt_supported(65536, 4096, 1024)
    x, w, _ = _mk(320, 256, 128)
    with pytest.raises(RuntimeError):
        hip.gemm_pnt(x, w)
