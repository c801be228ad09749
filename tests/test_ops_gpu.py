"""Numerics of every HIP kernel against a plain PyTorch fp32 reference.

Each test feeds the SAME bf16 inputs to the HIP op and to an fp32 reference
(autograd in fp32 for gradients) and bounds the error relative to the
reference's magnitude (bf16 output rounding ≈ 4e-3 relative).
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.fixture(autouse=True)
def _hip_mode(monkeypatch):
    monkeypatch.setenv("PDO_OPS", "hip")


def _ops():
    from paddle_operator_amd import _native, ops
    _native.require_hip()
    return ops


def test_extension_loaded(cuda):
    from paddle_operator_amd import _native
    m = _native.require_hip()
    assert m.arch == "gfx950"


@pytest.mark.parametrize("N,C", [(512, 1024), (300, 768), (64, 1600)])
def test_layernorm(cuda, N, C):
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(0)
    x = torch.randn(N, C, device=cuda, generator=g).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16().requires_grad_()
    y = ops.layer_norm(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    yf = torch.nn.functional.layer_norm(xf, (C,), wf, bf, 1e-5)
    yf.backward(dy.float())
    assert rel_err(y, yf) < 1e-2
    assert rel_err(x.grad, xf.grad) < 2e-2
    assert rel_err(w.grad, wf.grad) < 2e-2
    assert rel_err(b.grad, bf.grad) < 2e-2


@pytest.mark.parametrize("N,C,with_rb", [(1024, 1024, False), (16384, 1024, True), (333, 768, True)])
def test_add_layernorm(cuda, N, C, with_rb):
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(1)
    x = torch.randn(N, C, device=cuda, generator=g).bfloat16().requires_grad_()
    r = torch.randn(N, C, device=cuda, generator=g).bfloat16().requires_grad_()
    w = (1 + 0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16().requires_grad_()
    rb = (0.1 * torch.randn(C, device=cuda, generator=g)).bfloat16().requires_grad_() if with_rb else None
    h, y = ops.add_layer_norm(x, r, w, b, rbias=rb)
    dh, dy = torch.randn_like(h), torch.randn_like(y)
    torch.autograd.backward([h, y], [dh, dy])
    xf, rf, wf, bf = (t.detach().float().requires_grad_() for t in (x, r, w, b))
    rbf = rb.detach().float().requires_grad_() if with_rb else None
    hf = xf + rf + (rbf if with_rb else 0)
    yf = torch.nn.functional.layer_norm(hf, (C,), wf, bf, 1e-5)
    torch.autograd.backward([hf, yf], [dh.float(), dy.float()])
    assert rel_err(h, hf) < 1e-2
    assert rel_err(y, yf) < 1e-2
    assert rel_err(x.grad, xf.grad) < 2e-2
    assert rel_err(r.grad, rf.grad) < 2e-2
    assert rel_err(w.grad, wf.grad) < 2e-2
    assert rel_err(b.grad, bf.grad) < 2e-2
    if with_rb:
        assert rel_err(rb.grad, rbf.grad) < 2e-2


@pytest.mark.parametrize("R,C", [(64, 64), (1024, 4096), (4096, 1024), (50304, 1024), (192, 320)])
def test_transpose(cuda, R, C):
    ops = _ops()
    x = torch.randn(R, C, device=cuda).bfloat16()
    y = ops.transpose(x)
    assert y.shape == (C, R) and y.is_contiguous()
    assert torch.equal(y, x.t())  # a permutation: bitwise


@pytest.mark.parametrize("N,F", [(16384, 3072), (100, 1024)])
def test_bias_grad_and_linear(cuda, N, F):
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(11)
    K = 512
    x = torch.randn(N, K, device=cuda, generator=g).bfloat16().requires_grad_()
    w = (0.05 * torch.randn(F, K, device=cuda, generator=g)).bfloat16().requires_grad_()
    b = torch.randn(F, device=cuda, generator=g).bfloat16().requires_grad_()
    y = ops.linear(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    yf = torch.nn.functional.linear(xf, wf, bf)
    yf.backward(dy.float())
    assert rel_err(y, yf) < 2e-2
    assert rel_err(x.grad, xf.grad) < 2e-2
    assert rel_err(w.grad, wf.grad) < 2e-2
    assert rel_err(b.grad, bf.grad) < 2e-2


def test_linear_direct_arena_grad(cuda):
    """dW lands in the flat arena via addmm_ and the ready-callback fires once."""
    from paddle_operator_amd.parallel.flat import FlatParams
    from paddle_operator_amd import ops

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.randn(256, 128) * 0.05)
            self.b = torch.nn.Parameter(torch.zeros(256))

        def forward(self, x):
            return ops.linear(x, self.w, self.b)

    m = M().to(cuda).bfloat16()
    fp_ = FlatParams(m, device=cuda)
    seen = []
    m.w._pdo_ready = lambda p: seen.append(p)
    x = torch.randn(64, 128, device=cuda).bfloat16()
    for _ in range(2):  # two micro-batches accumulate
        m(x).float().sum().backward()
    assert len(seen) == 2
    ref = 2 * (torch.ones(64, 256, device=cuda).t() @ x.float())
    assert rel_err(m.w.grad, ref) < 2e-2
    assert m.w.grad.data_ptr() == fp_.grads[fp_.slots[[s.name for s in fp_.slots].index("w")].offset:].data_ptr()


@pytest.mark.parametrize("T,Fo,K", [(16384, 1024, 1024), (8192, 3072, 512)])
def test_linear_splitk_weight_grad(cuda, T, Fo, K):
    """Long-K dW takes the batched split-K path + HIP fold into the arena (accumulating)."""
    from paddle_operator_amd.parallel.flat import FlatParams
    from paddle_operator_amd import ops

    assert ops._splitk(T, Fo, K) > 1

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.randn(Fo, K) * 0.02)

        def forward(self, x):
            return ops.linear(x, self.w)

    m = M().to(cuda).bfloat16()
    FlatParams(m, device=cuda)
    g = torch.Generator(device=cuda).manual_seed(11)
    x = torch.randn(T, K, device=cuda, generator=g).bfloat16()
    dy = torch.randn(T, Fo, device=cuda, generator=g).bfloat16()
    for _ in range(2):
        m(x).backward(dy)
    ref = 2 * (dy.float().t() @ x.float())
    assert rel_err(m.w.grad, ref) < 2e-2


@pytest.mark.parametrize("T,M,N,acc", [(4096, 256, 512, False), (16384, 1024, 1024, True), (65536, 512, 256, True),
                                       (1024, 768, 256, False)])
def test_gemm_dw(cuda, T, M, N, acc):
    """HIP weight-gradient GEMM (token-major operands, transposing LDS reads, split-K) vs fp32."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    g = torch.Generator(device=cuda).manual_seed(13)
    dy = torch.randn(T, M, device=cuda, generator=g).bfloat16()
    x = torch.randn(T, N, device=cuda, generator=g).bfloat16()
    out = torch.randn(M, N, device=cuda, generator=g).bfloat16() if acc else torch.zeros(M, N, device=cuda).bfloat16()
    ref = out.float() + dy.float().t() @ x.float()
    assert m.gemm_dw(dy, x, out, True)
    assert rel_err(out, ref) < 1e-2, m.gemm_dw_splits(T, M, N)


def test_gemm_dw_rejects_unsupported_shape(cuda):
    from paddle_operator_amd import _native
    m = _native.require_hip()
    dy = torch.zeros(1000, 256, device=cuda).bfloat16()  # T % 64 != 0
    x = torch.zeros(1000, 256, device=cuda).bfloat16()
    assert m.gemm_dw_splits(1000, 256, 256) == 0
    assert not m.gemm_dw(dy, x, torch.zeros(256, 256, device=cuda).bfloat16(), True)


@pytest.mark.parametrize("T,Fo,K", [(32768, 4096, 4096), (8192, 640, 512)])
def test_linear_splitk_nondirect_weight_grad(cuda, T, Fo, K):
    """dW outside the arena (a fresh tensor for autograd, as for the tied LM head):
    gemm_dw (incl. a half-height last tile row) or split-K hipBLASLt."""
    from paddle_operator_amd import ops
    g = torch.Generator(device=cuda).manual_seed(12)
    w = (0.02 * torch.randn(Fo, K, device=cuda, generator=g)).bfloat16().requires_grad_()
    x = torch.randn(T, K, device=cuda, generator=g).bfloat16()
    dy = torch.randn(T, Fo, device=cuda, generator=g).bfloat16()
    ops.linear(x, w).backward(dy)
    assert rel_err(w.grad, dy.float().t() @ x.float()) < 2e-2


def test_arena_direct_norm_and_bias_grads(cuda):
    """LayerNorm γ/β, folded residual biases, bias-GELU and linear biases reduce
    straight into the flat arena (accumulating, no AccumulateGrad) and match fp32."""
    from paddle_operator_amd import ops
    from paddle_operator_amd.parallel.flat import FlatParams
    N, C = 2048, 1024
    torch.manual_seed(5)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w1 = torch.nn.Parameter(1 + 0.1 * torch.randn(C))
            self.b1 = torch.nn.Parameter(0.1 * torch.randn(C))
            self.w2 = torch.nn.Parameter(1 + 0.1 * torch.randn(C))
            self.b2 = torch.nn.Parameter(0.1 * torch.randn(C))
            self.rb = torch.nn.Parameter(0.1 * torch.randn(C))
            self.lw = torch.nn.Parameter(0.02 * torch.randn(C, C))
            self.lb = torch.nn.Parameter(0.1 * torch.randn(C))
            self.gb = torch.nn.Parameter(0.1 * torch.randn(C))

        def forward(self, x, r, hip=True):
            if hip:
                h = ops.layer_norm(x, self.w1, self.b1)
                _, y = ops.add_layer_norm(x, r + h, self.w2, self.b2, rbias=self.rb)
                return ops.bias_gelu(ops.linear(y, self.lw, self.lb), self.gb)
            F_ = torch.nn.functional
            h = F_.layer_norm(x, (C,), self.w1, self.b1)
            y = F_.layer_norm(x + r + h + self.rb, (C,), self.w2, self.b2)
            return ops.ref_bias_gelu(F_.linear(y, self.lw, self.lb), self.gb)

    m = M().to(cuda)
    ref = M().to(cuda)
    ref.load_state_dict(m.state_dict())
    m = m.bfloat16()
    FlatParams(m, device=cuda)
    g = torch.Generator(device=cuda).manual_seed(6)
    x = torch.randn(N, C, device=cuda, generator=g)
    r = torch.randn(N, C, device=cuda, generator=g)
    dy = torch.randn(N, C, device=cuda, generator=g)
    for _ in range(2):  # accumulates like two micro-batches
        m(x.bfloat16(), r.bfloat16()).backward(dy.bfloat16())
    for _ in range(2):
        ref(x, r, hip=False).backward(dy)
    for name, p in m.named_parameters():
        q = dict(ref.named_parameters())[name]
        assert rel_err(p.grad, q.grad) < 3e-2, name


@pytest.mark.parametrize("N,F", [(1024, 4096), (77, 3072)])
def test_bias_gelu(cuda, N, F):
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(2)
    x = (2 * torch.randn(N, F, device=cuda, generator=g)).bfloat16().requires_grad_()
    b = torch.randn(F, device=cuda, generator=g).bfloat16().requires_grad_()
    y = ops.bias_gelu(x, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xf, bf = (t.detach().float().requires_grad_() for t in (x, b))
    yf = torch.nn.functional.gelu(xf + bf, approximate="tanh")
    yf.backward(dy.float())
    assert rel_err(y, yf) < 1e-2
    assert rel_err(x.grad, xf.grad) < 2e-2
    assert rel_err(b.grad, bf.grad) < 2e-2


def test_cross_entropy(cuda):
    ops = _ops()
    N, V, Vp = 512, 50257, 50304
    g = torch.Generator(device=cuda).manual_seed(3)
    logits = (3 * torch.randn(N, Vp, device=cuda, generator=g)).bfloat16()
    logits[:, V:] = 100.0  # padding must be masked, even when huge
    tgt = torch.randint(0, V, (N,), device=cuda, generator=g)
    tgt[5] = -100  # ignored row
    lh = logits.clone().requires_grad_()
    loss = ops.cross_entropy(lh, tgt, V)
    loss.backward(torch.tensor(2.0, device=cuda))
    lf = logits.detach().float().requires_grad_()
    lossf = torch.nn.functional.cross_entropy(lf[:, :V], tgt, ignore_index=-100)
    (2.0 * lossf).backward()
    assert abs(loss.item() - lossf.item()) < 1e-3 * max(1.0, lossf.item())
    assert rel_err(lh.grad[:, :V], lf.grad[:, :V]) < 2e-2
    assert lh.grad[:, V:].abs().max().item() == 0.0
    assert lh.grad[5].abs().max().item() == 0.0


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("N,C,V,chunk", [(1024, 256, 1000, 256), (2048, 512, 50257, 512), (2048, 512, 50257, -1)])
def test_lm_head_xent_chunked(cuda, N, C, V, chunk, fused):
    """Chunked LM head + cross-entropy (ops._LMHeadXentFn) vs fp32 autograd:
    loss, dh and dW (incl. an ignored target, padded vocabulary rows, and the
    50304-row half-width last tile at V = 50257); chunk -1 = one chunk of every
    token; fused = the one-kernel statistics + dlogits pass (xent_fused)."""
    ops = _ops()
    prev_f = ops._XENT_FUSED[0]
    ops._XENT_FUSED[0] = fused
    Vp = (V + 127) // 128 * 128
    g = torch.Generator(device=cuda).manual_seed(9)
    h = torch.randn(N, C, device=cuda, generator=g).bfloat16()
    w = (0.05 * torch.randn(Vp, C, device=cuda, generator=g)).bfloat16()
    w[V:] = 0
    tgt = torch.randint(0, V, (N,), device=cuda, generator=g)
    tgt[3] = -100
    prev = ops._LM_CHUNK[0]
    ops._LM_CHUNK[0] = chunk
    try:
        hh = h.clone().requires_grad_()
        ww = w.clone().requires_grad_()
        loss = ops.lm_head_xent(hh, ww, tgt, V)
        loss.backward(torch.tensor(1.5, device=cuda))
    finally:
        ops._LM_CHUNK[0] = prev
        ops._XENT_FUSED[0] = prev_f
    hf = h.float().requires_grad_()
    wf = w.float().requires_grad_()
    lossf = torch.nn.functional.cross_entropy((hf @ wf.t())[:, :V], tgt, ignore_index=-100)
    (1.5 * lossf).backward()
    assert abs(loss.item() - lossf.item()) < 2e-3 * max(1.0, lossf.item())
    assert rel_err(hh.grad, hf.grad) < 3e-2
    assert rel_err(ww.grad[:V], wf.grad[:V]) < 3e-2
    # no_grad (validation loss): the loss-only path, same value
    ops._LM_CHUNK[0] = chunk
    try:
        with torch.no_grad():
            loss_ng = ops.lm_head_xent(hh, ww, tgt, V)
    finally:
        ops._LM_CHUNK[0] = prev
    assert abs(loss_ng.item() - lossf.item()) < 2e-3 * max(1.0, lossf.item())


def test_embedding(cuda):
    ops = _ops()
    B, S, C, Vp, P = 4, 128, 256, 1024, 256
    g = torch.Generator(device=cuda).manual_seed(4)
    idx = torch.randint(0, 1000, (B, S), device=cuda, generator=g)
    idx[0, :10] = 7  # repeated token → atomics collide
    wte = torch.randn(Vp, C, device=cuda, generator=g).bfloat16().requires_grad_()
    wpe = torch.randn(P, C, device=cuda, generator=g).bfloat16().requires_grad_()
    y = ops.embedding(idx, wte, wpe)
    dy = torch.randn_like(y)
    y.backward(dy)
    wf, pf = (t.detach().float().requires_grad_() for t in (wte, wpe))
    yf = torch.nn.functional.embedding(idx, wf) + pf[:S].unsqueeze(0)
    yf.backward(dy.float())
    assert rel_err(y, yf) < 1e-2
    assert rel_err(wte.grad, wf.grad) < 2e-2
    assert rel_err(wpe.grad, pf.grad) < 2e-2


def test_embedding_sorted_backward_into_arena(cuda):
    """The deterministic sorted segmented d(wte) (split tied weight: written
    straight into the gradient slot) equals the fp32-atomic table path, adds
    onto what the slot holds, and leaves rows of absent tokens untouched."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    B, S, C, Vp, P = 4, 128, 256, 1024, 256
    g = torch.Generator(device=cuda).manual_seed(14)
    idx = torch.randint(0, 300, (B, S), device=cuda, generator=g)
    idx[1, :40] = 5  # a long run of one token
    dy = torch.randn(B, S, C, device=cuda, generator=g).bfloat16()
    ref_wte, ref_wpe = m.embed_bwd(dy, idx, Vp, P)
    base = torch.randn(Vp, C, device=cuda, generator=g).bfloat16()
    slot = base.clone()
    keys, perm = torch.sort(idx.reshape(-1), stable=True)
    dwpe = m.embed_bwd_sorted(dy, keys, perm, slot, P)
    torch.testing.assert_close((slot.float() - base.float()), ref_wte.float(), atol=3e-2, rtol=2e-2)
    assert torch.equal(slot[300:], base[300:])  # tokens ≥ 300 never occur
    assert torch.equal(dwpe, ref_wpe)
    slot2 = base.clone()
    m.embed_bwd_sorted(dy, keys, perm, slot2, P)
    assert torch.equal(slot, slot2)  # deterministic


@pytest.mark.parametrize("skew", ["one_token", "runs_across_segments"])
def test_embedding_sorted_backward_skewed_ids(cuda, skew):
    """Skewed token ids (a frequent EOS/padding id): runs of equal ids longer
    than the 256-row segments of the sorted embedding backward are summed in
    pieces and folded in segment order — against an fp32 index_add reference,
    deterministic, ids outside the table ignored."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    B, S, C, Vp, P = 16, 512, 256, 1024, 512
    g = torch.Generator(device=cuda).manual_seed(21)
    idx = torch.randint(0, 900, (B, S), device=cuda, generator=g)
    if skew == "one_token":
        idx[torch.rand(B, S, device=cuda, generator=g) < 0.7] = 3  # 70 %: ~5700 rows of one id
    else:
        idx.view(-1)[:1000] = 11        # runs crossing 3 segment boundaries
        idx.view(-1)[1000:1300] = 12
        idx[-1, -20:] = Vp + 5          # outside the table: contributes nothing
    dy = torch.randn(B, S, C, device=cuda, generator=g).bfloat16()
    keys, perm = torch.sort(idx.reshape(-1), stable=True)
    base = torch.randn(Vp, C, device=cuda, generator=g).bfloat16()
    slot = base.clone()
    m.embed_bwd_sorted(dy, keys, perm, slot, P)
    ok = idx.reshape(-1) < Vp
    ref = torch.zeros(Vp, C, device=cuda).index_add_(0, idx.reshape(-1)[ok], dy.reshape(-1, C)[ok].float())
    torch.testing.assert_close(slot.float(), base.float() + ref, atol=5e-2, rtol=1e-2)
    slot2 = base.clone()
    m.embed_bwd_sorted(dy, keys, perm, slot2, P)
    assert torch.equal(slot, slot2)


def test_sgd_flat_matches_reference(cuda):
    """The fused momentum-SGD pass (ResNet-50's optimizer) equals the bulk-op formula."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    n = 64 * 1024
    g_ = torch.Generator(device=cuda).manual_seed(15)
    w = torch.randn(n, device=cuda, generator=g_)
    g = torch.randn(n, device=cuda, generator=g_)
    buf = torch.randn(n, device=cuda, generator=g_)
    decay = (torch.rand(n // 1024, device=cuda, generator=g_) > 0.5).float()
    lr, mom, wd, sc = 0.1, 0.9, 5e-5, 0.25
    dec = decay.repeat_interleave(1024)
    ref_b = mom * buf + (g * sc + wd * dec * w)
    ref_w = w - lr * ref_b
    m.sgd_flat(w, g, buf, decay, lr, mom, wd, sc)
    torch.testing.assert_close(buf, ref_b, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(w, ref_w, rtol=1e-6, atol=1e-6)


def _attn_ref(qkv, H):
    B, S, C3 = qkv.shape
    C = C3 // 3
    D = C // H
    qf = qkv.detach().float().requires_grad_()
    q, k, v = qf.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)
    s = q @ k.transpose(-1, -2) / math.sqrt(D)
    mask = torch.ones(S, S, dtype=torch.bool, device=qkv.device).triu(1)
    p = torch.softmax(s.masked_fill(mask, float("-inf")), dim=-1)
    o = (p @ v).transpose(1, 2).reshape(B, S, C)
    return qf, o


@pytest.mark.parametrize("B,S,H", [(2, 256, 2), (1, 1024, 4), (3, 128, 1)])
def test_attention(cuda, B, S, H):
    ops = _ops()
    D = 64
    g = torch.Generator(device=cuda).manual_seed(5)
    qkv = torch.randn(B, S, 3 * H * D, device=cuda, generator=g).bfloat16().requires_grad_()
    o = ops.attention(qkv, H)
    do = torch.randn_like(o)
    o.backward(do)
    qf, of = _attn_ref(qkv, H)
    of.backward(do.float())
    assert rel_err(o, of) < 2e-2
    dq = qkv.grad.view(B, S, 3, H * D)
    dqf = qf.grad.view(B, S, 3, H * D)
    for i, name in enumerate("qkv"):
        e = rel_err(dq[:, :, i], dqf[:, :, i])
        assert e < 3e-2, f"d{name} rel err {e}"


def test_attention_forced_rescale(cuda):
    """Spike one key so the running max jumps mid-sequence (online-softmax
    rescale branch must be exact: cdna_hip_programming.md §5.4 rule 26)."""
    ops = _ops()
    B, S, H, D = 1, 512, 1, 64
    g = torch.Generator(device=cuda).manual_seed(6)
    qkv = torch.randn(B, S, 3 * H * D, device=cuda, generator=g)
    qkv[0, :, :D] = 0.5  # all queries equal
    qkv[0, 300, D:2 * D] = 8.0  # key 300 dominates for queries >= 300
    qkv = qkv.bfloat16().requires_grad_()
    o = ops.attention(qkv, H)
    qf, of = _attn_ref(qkv, H)
    assert rel_err(o, of) < 2e-2


def test_grad_norm_chunks_order_independent(cuda):
    """Global-norm partials per fixed chunk (csrc/hip/optim.hip sumsq_chunks):
    taken in bucket-sized pieces or in one pass, the same bits; against fp64."""
    from paddle_operator_amd.ops.optim import FlatAdamW
    from paddle_operator_amd.parallel.flat import FlatParams
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(1024, 1000), torch.nn.Linear(1000, 700)).to(cuda).bfloat16()
    fp_ = FlatParams(net, device=cuda)
    opt = FlatAdamW(fp_, lr=1e-2, max_grad_norm=0.5, norm_chunk=1 << 16)
    assert opt._norm_part.numel() > 20
    fp_.grads.copy_(torch.randn_like(fp_.grads.float()).bfloat16())
    one = opt.grad_norm_sq(0.5).clone()
    opt.norm_reset()
    for upto in (70_000, 70_001, 300_000, 900_000, 1_000_000):  # bucket ends, not chunk-aligned
        opt.norm_partial(upto)
    split = opt.grad_norm_sq(0.5).clone()
    assert torch.equal(one, split)
    ref = (fp_.param_grads.double() * 0.5).pow(2).sum()
    assert abs(float(one) - float(ref)) / float(ref) < 1e-5


def test_adamw_matches_reference(cuda):
    from paddle_operator_amd.ops.optim import FlatAdamW
    from paddle_operator_amd.parallel.flat import FlatParams
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 8)).to(cuda).bfloat16()
    fp_ = FlatParams(net, device=cuda)
    opt = FlatAdamW(fp_, lr=1e-2, max_grad_norm=0.5)
    fp_.grads.copy_(torch.randn_like(fp_.grads.float()).bfloat16())
    # reference: same math through the torch path
    master0, g0 = opt.master.clone(), fp_.grads.float().clone()
    opt.step(grad_scale=0.5)
    import os
    os.environ["PDO_OPS"] = "torch"
    try:
        ref = FlatAdamW.__new__(FlatAdamW)
        ref.__dict__.update(opt.__dict__)
        ref.master = master0
        ref.m = torch.zeros_like(master0)
        ref.v = torch.zeros_like(master0)
        ref.step_count = 0
        ref._norm_buf = torch.zeros(2, device=cuda)
        params_before = fp_.params.clone()
        ref.flat = type("F", (), {})()
        ref.flat.grads = g0.bfloat16()
        ref.flat.param_grads = ref.flat.grads
        ref.flat.params = params_before
        ref.flat.decay_chunks = fp_.decay_chunks
        ref.flat.numel = fp_.numel
        ref.flat.device = fp_.device
        ref.step(grad_scale=0.5)
    finally:
        os.environ["PDO_OPS"] = "hip"
    assert rel_err(opt.master, ref.master) < 1e-5
    assert rel_err(opt.m, ref.m) < 1e-5
    assert rel_err(opt.v, ref.v) < 1e-5


def test_gpt2_tiny_hip_vs_torch(cuda):
    """Whole-model forward/backward: HIP ops vs torch ops on the same weights."""
    import os
    from paddle_operator_amd.models.gpt2 import GPT2, GPT2Config
    cfg = GPT2Config.named("gpt2-tiny")
    torch.manual_seed(0)
    m = GPT2(cfg).to(cuda).bfloat16()
    idx = torch.randint(0, cfg.vocab_size, (2, 257), device=cuda)
    x, y = idx[:, :-1], idx[:, 1:]
    loss_h = m(x, y)
    loss_h.backward()
    gh = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    os.environ["PDO_OPS"] = "torch"
    try:
        loss_t = m(x, y)
        loss_t.backward()
    finally:
        os.environ["PDO_OPS"] = "hip"
    assert abs(loss_h.item() - loss_t.item()) < 2e-2
    for n, p in m.named_parameters():
        assert rel_err(gh[n], p.grad) < 6e-2, n


@pytest.mark.gpu
def test_gpt2_medium_width_hip_vs_fp32(cuda):
    """Two layers at GPT-2-medium width — C = 1024, 16 heads, vocab 50304,
    S = 1024, B = 8 (8192 tokens): every GEMM, attention, LayerNorm and
    cross-entropy kernel at the production shape except the token count.  The
    HIP path in bf16 against the SAME weights in fp32 with the plain torch ops:
    the loss and every parameter gradient."""
    import copy
    import os
    from paddle_operator_amd.models.gpt2 import GPT2, GPT2Config
    cfg = GPT2Config(n_embd=1024, n_layer=2, n_head=16)
    with torch.device(cuda):
        ref = GPT2(cfg)  # fp32, initialised on the device
    m = copy.deepcopy(ref).bfloat16()
    g = torch.Generator(device=cuda).manual_seed(5)
    idx = torch.randint(0, cfg.vocab_size, (8, 1025), device=cuda, generator=g)
    x, y = idx[:, :-1], idx[:, 1:]
    loss_h = m(x, y)
    loss_h.backward()
    os.environ["PDO_OPS"] = "torch"
    try:
        loss_r = ref(x, y)
        loss_r.backward()
    finally:
        os.environ["PDO_OPS"] = "hip"
    assert abs(loss_h.item() - loss_r.item()) < 2e-2, (loss_h.item(), loss_r.item())
    errs = {n: rel_err(p.grad, dict(ref.named_parameters())[n].grad) for n, p in m.named_parameters()}
    bad = {n: e for n, e in errs.items() if not e < 5e-2}
    assert not bad, bad


@pytest.mark.gpu
def test_qkv_attention_fused_bias_grad(cuda):
    """QKV projection + attention node (bias gradient from the attention kernels'
    column partials) == separate linear + attention nodes, and ≈ fp32."""
    ops = _ops()
    B, S, H, C = 2, 256, 4, 256
    g = torch.Generator(device=cuda).manual_seed(21)
    base = [torch.randn(B, S, C, device=cuda, generator=g).bfloat16(),
            (0.05 * torch.randn(3 * C, C, device=cuda, generator=g)).bfloat16(),
            (0.1 * torch.randn(3 * C, device=cuda, generator=g)).bfloat16()]
    do = torch.randn(B, S, C, device=cuda, generator=g).bfloat16()
    grads = []
    for fused in (True, False):
        ops._QKV_FUSED[0] = fused
        try:
            ts = [t.clone().requires_grad_() for t in base]
            ops.qkv_attention(ts[0], ts[1], ts[2], H).backward(do)
        finally:
            ops._QKV_FUSED[0] = True
        grads.append([t.grad.float() for t in ts])
    for a, b, name in zip(grads[0], grads[1], ("dh", "dw", "db")):
        assert rel_err(a, b) < 1e-2, name
    ref = [t.detach().float().requires_grad_() for t in base]
    qkv = ref[0] @ ref[1].t() + ref[2]
    q, k, v = qkv.view(B, S, 3, H, C // H).permute(2, 0, 3, 1, 4).unbind(0)
    o = ops.ref_attention(q, k, v, causal=True).transpose(1, 2).reshape(B, S, C)
    o.backward(do.float())
    assert rel_err(grads[0][2], ref[2].grad) < 3e-2


@pytest.mark.gpu
@pytest.mark.parametrize("nt_gelu,saved_grad", [(True, True), (True, False), (False, False)])
def test_mlp_nt_dgelu_matches_unfused(cuda, nt_gelu, saved_grad):
    """gemm_nt epilogues in the MLP — fc1 GELU forward (_NTMLPFn, saving gelu' or
    the pre-activation) and/or fc2's input gradient ⊙ GELU' — == hipBLASLt + the
    bias-GELU kernels (output and every gradient)."""
    ops = _ops()
    ops._NT_GD[0] = saved_grad
    T, C = 4096, 512
    g = torch.Generator(device=cuda).manual_seed(5)
    base = [(0.05 * torch.randn(T, C, device=cuda, generator=g)).bfloat16() * 20,
            (0.05 * torch.randn(4 * C, C, device=cuda, generator=g)).bfloat16(),
            (0.1 * torch.randn(4 * C, device=cuda, generator=g)).bfloat16(),
            (0.05 * torch.randn(C, 4 * C, device=cuda, generator=g)).bfloat16()]
    dy = torch.randn(T, C, device=cuda, generator=g).bfloat16()
    grads, outs = [], []
    for fused in (True, False):
        ops._NT_DGELU[0] = fused
        ops._NT_GELU[0] = fused and nt_gelu
        try:
            ts = [t.clone().requires_grad_() for t in base]
            y = ops.mlp(*ts)
            y.backward(dy)
        finally:
            ops._NT_DGELU[0] = True
            ops._NT_GELU[0] = True
            ops._NT_GD[0] = True
        outs.append(y.detach().float())
        grads.append([t.grad.float() for t in ts])
    assert rel_err(outs[0], outs[1]) < 1e-2, "y"
    for a, b, name in zip(grads[0], grads[1], ("dx", "dw1", "db1", "dw2")):
        assert rel_err(a, b) < 1e-2, name


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,relu,res", [(8, 64, 28, True, False), (4, 256, 14, True, True),
                                              (16, 128, 7, False, False), (2, 2048, 7, True, True),
                                              (4, 24, 9, True, False), (3, 40, 5, True, True)])
def test_bn_act_nhwc(cuda, N, C, H, relu, res):
    """Fused NHWC BatchNorm(+residual)(+ReLU) vs fp32 PyTorch, incl. running stats."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(13)
    x = (3 + 2 * torch.randn(N, C, H, H, device=cuda, generator=g)).bfloat16()
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_()
    r = None
    if res:
        r = torch.randn(N, C, H, H, device=cuda, generator=g).bfloat16()
        r = r.contiguous(memory_format=torch.channels_last).requires_grad_()
    bn = torch.nn.BatchNorm2d(C).to(cuda)
    with torch.no_grad():
        bn.weight.copy_(1 + 0.1 * torch.randn(C, device=cuda, generator=g))
        bn.bias.copy_(0.1 * torch.randn(C, device=cuda, generator=g))
    bnf = torch.nn.BatchNorm2d(C).to(cuda)
    bnf.load_state_dict(bn.state_dict())
    y = ops.bn_act(bn, x, relu=relu, residual=r)
    dy = torch.randn_like(y)
    y.backward(dy)
    xf = x.detach().float().requires_grad_()
    rf = r.detach().float().requires_grad_() if res else None
    yf = bnf(xf)
    if res:
        yf = yf + rf
    if relu:
        yf = torch.relu(yf)
    yf.backward(dy.float())
    assert rel_err(y, yf) < 2e-2
    assert rel_err(x.grad, xf.grad) < 3e-2
    assert rel_err(bn.weight.grad, bnf.weight.grad) < 2e-2
    assert rel_err(bn.bias.grad, bnf.bias.grad) < 2e-2
    if res:
        assert rel_err(r.grad, rf.grad) < 2e-2
    assert rel_err(bn.running_mean, bnf.running_mean) < 1e-3
    assert rel_err(bn.running_var, bnf.running_var) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("N,Cin,Cout,H", [(16, 256, 64, 16), (16, 64, 256, 16), (8, 512, 256, 16),
                                          (16, 1024, 256, 8), (4, 64, 64, 16), (8, 256, 128, 32)])
def test_conv1x1_gemm_path_vs_fp32(cuda, N, Cin, Cout, H):
    """ops.conv1x1 (GEMM products, MIOpen where it measured faster) against an
    fp32 convolution: output, input gradient and weight gradient, under
    autocast with an fp32 master weight as in the ResNet trainer."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(Cin + Cout)
    conv = torch.nn.Conv2d(Cin, Cout, 1, bias=False).to(cuda)
    with torch.no_grad():
        conv.weight.copy_(0.05 * torch.randn(conv.weight.shape, device=cuda, generator=g))
    x = torch.randn(N, Cin, H, H, device=cuda, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(N, Cout, H, H, device=cuda, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    xh = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops.conv1x1(conv, xh)
    y.backward(dy)
    assert y.is_contiguous(memory_format=torch.channels_last)
    xf = x.float().requires_grad_()
    wf = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    yf = torch.nn.functional.conv2d(xf, wf)
    yf.backward(dy.float())
    assert rel_err(y, yf) < 1e-2
    assert rel_err(xh.grad, xf.grad) < 1e-2
    assert conv.weight.grad.dtype == torch.float32
    assert rel_err(conv.weight.grad, wf.grad) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,W", [(4, 64, 112, 112), (2, 16, 9, 7), (3, 8, 2, 5)])
def test_maxpool3s2_nhwc(cuda, N, C, H, W):
    """HIP 3×3/2 max-pool (fwd value + gather backward) vs fp32 PyTorch."""
    ops = _ops()
    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(N, C, H, W, device=cuda, generator=g).bfloat16()
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_()
    y = ops.max_pool_3x3s2(x)
    xf = x.detach().float().requires_grad_()
    yf = torch.nn.functional.max_pool2d(xf, 3, 2, 1)
    assert y.shape == yf.shape
    assert torch.equal(y.float(), yf)
    dy = torch.randn(y.shape, device=cuda, generator=g).bfloat16()
    y.backward(dy)
    yf.backward(dy.float())
    assert rel_err(x.grad, xf.grad) < 1e-2


@pytest.mark.parametrize("T,M,N,acc,splits", [(8192, 384, 512, True, 0), (8192, 384, 512, False, 1),
                                              (16384, 2944, 256, True, 0), (4096, 640, 768, True, 2)])
def test_gemm_dw4_half_height_edge(cuda, T, M, N, acc, splits):
    """M % 256 == 128 (the LM head's 50304-row vocabulary): gemm_dw4's half-height last
    tile row — its missing A columns re-fetched in bounds, its rows never stored."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    g = torch.Generator(device=cuda).manual_seed(23)
    dy = torch.empty(T, M, device=cuda).uniform_(-1, 1, generator=g).bfloat16()
    x = torch.empty(T, N, device=cuda).uniform_(-1, 1, generator=g).bfloat16()
    base = torch.empty(M, N, device=cuda).uniform_(-4, 4, generator=g).bfloat16() if acc else \
        torch.zeros(M, N, device=cuda).bfloat16()
    ref = base.float() + dy.float().t() @ x.float()
    prev = m.gemm_dw_impl(-1)
    try:
        for impl in (1, 2):
            m.gemm_dw_impl(impl)
            out = base.clone()
            assert m.gemm_dw(dy, x, out, True, splits)
            assert rel_err(out, ref) < 1e-2, (impl, splits, m.gemm_dw_splits(T, M, N))
        m.gemm_dw_impl(0)  # the 8-wave loop has no edge tile: unsupported, never wrong
        assert not m.gemm_dw(dy, x, base.clone(), True) or M % 256 == 0
    finally:
        m.gemm_dw_impl(prev)


@pytest.mark.parametrize("T,M,N,acc", [(8192, 4096, 4096, True), (65536, 1024, 3072, False), (16384, 512, 768, True),
                                       (16384, 3072, 1024, True)])  # last: 48 tiles → 5 uneven slices
def test_gemm_dw_mainloops_agree(cuda, T, M, N, acc):
    """The 4-wave dW mainloop (gemm_dw4.hip, both schedules: 16x16x32 and 32x32x16 MFMAs; split-K or
    in-kernel accumulate at one split) and the 8-wave one against fp32."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    g = torch.Generator(device=cuda).manual_seed(21)
    dy = torch.empty(T, M, device=cuda).uniform_(-1, 1, generator=g).bfloat16()
    x = torch.empty(T, N, device=cuda).uniform_(-1, 1, generator=g).bfloat16()
    base = torch.empty(M, N, device=cuda).uniform_(-4, 4, generator=g).bfloat16() if acc else \
        torch.zeros(M, N, device=cuda).bfloat16()
    ref = base.float() + dy.float().t() @ x.float()
    prev = m.gemm_dw_impl(0)
    try:
        for impl in (0, 1, 2):
            m.gemm_dw_impl(impl)
            out = base.clone()
            assert m.gemm_dw(dy, x, out, True)
            assert rel_err(out, ref) < 1e-2, (impl, m.gemm_dw_splits(T, M, N))
    finally:
        m.gemm_dw_impl(prev)


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,K", [(4096, 1024, 1024), (2048, 512, 4096), (1024, 256, 128)])
def test_gemm_nt_add_bias(cuda, T, N, K):
    """c = a·bᵀ + bias + r (gemm_nt EPI 5) on the 4-wave mainloop (K ≥ 256) and
    the 8-wave ring (K = 128) against fp32."""
    from paddle_operator_amd import _native
    m = _native.require_hip()
    g = torch.Generator(device=cuda).manual_seed(T + K)
    a = torch.randn(T, K, device=cuda, generator=g).bfloat16()
    b = (torch.randn(N, K, device=cuda, generator=g) / K ** 0.5).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g).bfloat16()
    r = torch.randn(T, N, device=cuda, generator=g).bfloat16()
    c = m.gemm_nt_add(a, b, r, bias=bias)
    assert rel_err(c, a.float() @ b.float().t() + bias.float() + r.float()) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["proj", "mlp"])
def test_residual_epilogue_layernorm_matches_unfused(cuda, which):
    """The residual stream joined inside the output projection's GEMM epilogue
    (bias + x added there, a one-input LayerNorm after: ops.linear_add_layer_norm
    / ops.mlp_add_layer_norm) == the GEMM + fused add+LayerNorm path, for (h, y)
    and every input / parameter gradient."""
    ops = _ops()
    T, C = 4096, 512
    g = torch.Generator(device=cuda).manual_seed(11)
    mk = lambda *s, sc=1.0: (sc * torch.randn(*s, device=cuda, generator=g)).bfloat16()  # noqa: E731
    if which == "proj":
        base = [mk(T, C), mk(C, C, sc=0.05), mk(C, sc=0.1), mk(T, C), 1 + mk(C, sc=0.1), mk(C, sc=0.1)]
        fn = ops.linear_add_layer_norm
    else:
        base = [mk(T, C), mk(4 * C, C, sc=0.05), mk(4 * C, sc=0.1), mk(C, 4 * C, sc=0.05), mk(C, sc=0.1),
                mk(T, C), 1 + mk(C, sc=0.1), mk(C, sc=0.1)]
        fn = ops.mlp_add_layer_norm
    dh, dy = mk(T, C), mk(T, C)
    outs, grads = [], []
    for fused in (True, False):
        ops._RES_EPI[0] = fused
        try:
            ts = [t.clone().requires_grad_() for t in base]
            h, y = fn(*ts)
            torch.autograd.backward([h, y], [dh, dy])
        finally:
            ops._RES_EPI[0] = True
        outs.append((h.detach().float(), y.detach().float()))
        grads.append([t.grad.float() for t in ts])
    assert rel_err(outs[0][0], outs[1][0]) < 1e-2 and rel_err(outs[0][1], outs[1][1]) < 1e-2
    for i, (a, b) in enumerate(zip(grads[0], grads[1])):
        assert rel_err(a, b) < 2e-2, i
