"""CPU checks of model-level rewrites the HIP kernels rely on."""
import torch
import torch.nn.functional as F


def _s2d(x):
    """[N, 3, H, W] → the stem's 16-channel image [N, 16, H/2, W/2]:
    z[n, (2p + q)·3 + c, i, j] = x[n, c, 2i + p, 2j + q], channels 12-15 zero
    (csrc/hip/conv.hip stem_s2d_kernel)."""
    N, C, H, W = x.shape
    z = x.view(N, C, H // 2, 2, W // 2, 2).permute(0, 3, 5, 1, 2, 4).reshape(N, 4 * C, H // 2, W // 2)
    return F.pad(z, (0, 0, 0, 0, 0, 16 - 4 * C))


def _w2(w):
    """[K, 3, 7, 7] → [K, 16, 4, 4]: w8 = w padded to 8 × 8 at the top / left,
    w2[k, (2p + q)·3 + c, a, b] = w8[k, c, 2a + p, 2b + q] (stem_weight_kernel)."""
    K, C = w.shape[:2]
    w8 = F.pad(w, (1, 0, 1, 0)).view(K, C, 4, 2, 4, 2)
    return F.pad(w8.permute(0, 3, 5, 1, 2, 4).reshape(K, 4 * C, 4, 4), (0, 0, 0, 0, 0, 16 - 4 * C))


def test_stem_space_to_depth_identity():
    """conv7×7/2 pad 3 (x, w) = conv4×4/1 (z padded 2 before / 1 after, w2):
    the identity behind ops._StemFn, for even and odd half-sizes."""
    g = torch.Generator().manual_seed(0)
    for H, W in ((224, 224), (30, 30), (8, 14)):
        x = torch.randn(2, 3, H, W, generator=g, dtype=torch.float64)
        w = torch.randn(64, 3, 7, 7, generator=g, dtype=torch.float64)
        ref = F.conv2d(x, w, stride=2, padding=3)
        y = F.conv2d(F.pad(_s2d(x), (2, 1, 2, 1)), _w2(w))
        assert y.shape == ref.shape
        torch.testing.assert_close(y, ref, rtol=1e-10, atol=1e-10)
        # and its weight gradient maps back through the same permutation
        wf = w.clone().requires_grad_()
        F.conv2d(x, wf, stride=2, padding=3).backward(torch.ones_like(ref))
        w2 = _w2(w).requires_grad_()
        F.conv2d(F.pad(_s2d(x), (2, 1, 2, 1)), w2).backward(torch.ones_like(ref))
        d8 = w2.grad[:, :12].view(64, 2, 2, 3, 4, 4).permute(0, 3, 4, 1, 5, 2).reshape(64, 3, 8, 8)
        torch.testing.assert_close(d8[:, :, 1:, 1:], wf.grad, rtol=1e-10, atol=1e-8)


def test_residual_mask_link_hand_off_semantics():
    """ops._ResMaskLink: a given (dy, mask) is taken only by that exact gradient
    tensor (same storage, same version); anything else raises instead of being
    silently masked; an empty link takes nothing."""
    import pytest

    from paddle_operator_amd import ops

    link = ops._ResMaskLink()
    assert link.take(torch.zeros(4)) is None  # nothing given: no-op
    dy = torch.randn(2, 8)
    mask = torch.ones(2, dtype=torch.uint8)
    link.give(dy, mask)
    assert link.take(dy) is mask
    assert link.take(dy) is None  # consumed
    link.give(dy, mask)
    with pytest.raises(RuntimeError):
        link.take(dy.clone())  # another tensor: something was added to the gradient
    link.give(dy, mask)
    dy.add_(1.0)  # modified in place after the hand-off
    with pytest.raises(RuntimeError):
        link.take(dy)


def test_compact_grad_link_accumulates_and_clears():
    from paddle_operator_amd import ops

    link = ops._CompactGradLink()
    assert link.take() is None
    a, b = torch.ones(2, 3), torch.full((2, 3), 2.0)
    link.give(a)
    link.give(b)  # two compact contributions sum
    t = link.take()
    assert torch.equal(t, torch.full((2, 3), 3.0))
    assert link.take() is None


def test_apply_bitmask_matches_unpacked_mask():
    """ops._apply_bitmask on a channels_last tensor: bit j of byte i keeps element
    8i + j of the NHWC-flattened tensor (bn_apply_kernel's mask layout)."""
    from paddle_operator_amd import ops

    g = torch.Generator().manual_seed(1)
    t = torch.randn(2, 16, 3, 5, generator=g).contiguous(memory_format=torch.channels_last)
    mask = torch.randint(0, 256, (t.numel() // 8,), generator=g).to(torch.uint8)
    keep = ((mask.view(-1, 1) >> torch.arange(8, dtype=torch.uint8)) & 1).view(-1).float()
    ref = (t.permute(0, 2, 3, 1).reshape(-1) * keep).view(2, 3, 5, 16).permute(0, 3, 1, 2)
    assert torch.equal(ops._apply_bitmask(t, mask), ref)
