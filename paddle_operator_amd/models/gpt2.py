"""GPT-2 family (BASELINE config 4: GPT-2-medium, collective mode, 8×MI355X).

Architecture follows the public GPT-2 definition (pre-LN transformer, learned
positions, tanh-GELU MLP, tied input/output embedding).  Layout decisions are
MI355X-first rather than a transcription of any reference implementation:

* the vocabulary is padded 50257 → 50304 (a multiple of 128) so the LM-head
  GEMM tiles evenly on the 256-CU grid; padded logits are masked inside the
  fused cross-entropy kernel, so the loss is exactly the 50257-way loss;
* QKV stays packed ([B, S, 3, H, D]) and the flash-attention kernel reads it in
  place — no transpose/contiguous copies around attention;
* the attention output projection and fc2 add their bias and the residual
  stream in the GEMM epilogue, so the next LayerNorm reads the stream once
  (ops.linear_add_layer_norm / ops.mlp_add_layer_norm); bias + GELU and GELU'
  run in the fc1 / fc2 GEMM epilogues; embedding gather + position add is one
  kernel;
* every dense projection (forward, input gradient, weight gradient, LM head)
  runs on the hand-written gemm_nt4 / gemm_dw4 kernels; library GEMMs run
  only for shapes outside their contracts.

The reference operator has no model code at all; this workload
is what a PaddleJob launches (``deploy/examples/resnet.yaml:14-19`` pattern).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn

from .. import ops


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 1024
    n_layer: int = 24
    n_head: int = 16
    ln_eps: float = 1e-5
    # 128: 50304 rows.  256 (PDO_PAD_VOCAB=256): 50432, full 256-wide tiles, so the
    # LM head's forward / dX GEMMs enter gemm_nt4 and its dW gemm_dw4's full-height tiles
    pad_vocab_to: int = field(default_factory=lambda: int(os.environ.get("PDO_PAD_VOCAB", "128")))

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_to
        return (self.vocab_size + m - 1) // m * m

    @staticmethod
    def named(name: str) -> "GPT2Config":
        table = {
            "gpt2": dict(n_embd=768, n_layer=12, n_head=12),
            "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
            "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
            "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),
            # tiny config for CPU tests
            "gpt2-tiny": dict(n_embd=128, n_layer=2, n_head=2, n_positions=256, vocab_size=1000),
            # GPU smoke: the smallest width whose GEMMs (K = 256, 1024) enter the
            # hand-written gemm_nt4 / gemm_dw4 kernels, not their fallbacks
            "gpt2-smoke": dict(n_embd=256, n_layer=2, n_head=4, n_positions=512, vocab_size=4000),
        }
        return GPT2Config(**table[name])

    def n_params(self) -> int:
        C, L = self.n_embd, self.n_layer
        per_layer = 12 * C * C + 13 * C
        return self.padded_vocab * C + self.n_positions * C + L * per_layer + 2 * C

    def flops_per_token(self, seq: int) -> float:
        """Training FLOPs/token (fwd+bwd = 3× fwd), dense + attention."""
        C, L = self.n_embd, self.n_layer
        dense = 6 * (L * 12 * C * C + self.padded_vocab * C)
        attn = 6 * L * seq * C  # causal: QK^T and PV over on average S/2 keys (×2 matmuls)
        return float(dense + attn)


class Linear(nn.Module):
    """y = x @ W^T (+ b). Weight stored [out, in] like nn.Linear."""

    def __init__(self, fin, fout, bias=True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(fout, fin))
        self.bias = nn.Parameter(torch.zeros(fout)) if bias else None

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias)

    def forward_nobias(self, x):
        """Bias is applied by the consumer (fused into GELU / residual+LN)."""
        return ops.linear(x, self.weight)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        C = cfg.n_embd
        self.cfg = cfg
        self.ln1_w = nn.Parameter(torch.ones(C))
        self.ln1_b = nn.Parameter(torch.zeros(C))
        self.qkv = Linear(C, 3 * C)
        self.proj = Linear(C, C)
        self.ln2_w = nn.Parameter(torch.ones(C))
        self.ln2_b = nn.Parameter(torch.zeros(C))
        self.fc = Linear(C, 4 * C)
        self.fc_proj = Linear(4 * C, C)

    def forward(self, x, h, ln_next_w, ln_next_b):
        """x: residual stream, h: LN1(x) already computed by the caller.

        Returns (x_out, LN_next(x_out)) — the next block's LN1 (or the final LN)
        taken here, so each branch output joins the residual stream inside its
        output projection's GEMM epilogue (bias and residual added there,
        ops.linear_add_layer_norm / ops.mlp_add_layer_norm) and the following
        LayerNorm reads the stream once.
        """
        cfg = self.cfg
        a = ops.qkv_attention(h, self.qkv.weight, self.qkv.bias, cfg.n_head)
        x, h2 = ops.linear_add_layer_norm(a, self.proj.weight, self.proj.bias, x, self.ln2_w, self.ln2_b,
                                          cfg.ln_eps)
        return ops.mlp_add_layer_norm(h2, self.fc.weight, self.fc.bias, self.fc_proj.weight, self.fc_proj.bias,
                                      x, ln_next_w, ln_next_b, cfg.ln_eps)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        C = cfg.n_embd
        self.wte = nn.Parameter(torch.empty(cfg.padded_vocab, C))
        self.wpe = nn.Parameter(torch.empty(cfg.n_positions, C))
        self.blocks = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.lnf_w = nn.Parameter(torch.ones(C))
        self.lnf_b = nn.Parameter(torch.zeros(C))
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self, seed: int = 1234):
        """N(0, 0.02) weights (residual projections scaled by 1/sqrt(2·layers)).

        Parameters already on a GPU (the trainer builds the model under
        ``torch.device("cuda")``) are drawn in place by the device's generator:
        no host RNG over 355 M values and no host→device copy — the largest term
        of a GPT-2-medium rank's create→ready time (2.6 s in BENCH_r02, ≈2 s of
        it CPU randn).  On CPU the host generator keeps the reference stream."""
        dev = next(self.parameters()).device
        g = torch.Generator(device=dev).manual_seed(seed)
        std = 0.02
        proj_std = 0.02 / math.sqrt(2 * self.cfg.n_layer)
        for name, p in self.named_parameters():
            if p.dim() == 2:
                s = proj_std if (name.endswith("proj.weight") and "blocks" in name) else std
                if dev.type == "cpu":
                    p.copy_(torch.randn(p.shape, generator=g) * s)
                else:
                    p.normal_(0.0, s, generator=g)
        self.wte[self.cfg.vocab_size:].zero_()

    def forward(self, idx, targets=None):
        cfg = self.cfg
        x = ops.embedding(idx, self.wte, self.wpe)
        blk0 = self.blocks[0]
        x, h = ops.layer_norm_res(x, blk0.ln1_w, blk0.ln1_b, cfg.ln_eps)
        for i, blk in enumerate(self.blocks):
            if i + 1 < len(self.blocks):
                nb = self.blocks[i + 1]
                x, h = blk(x, h, nb.ln1_w, nb.ln1_b)
            else:
                x, h = blk(x, h, self.lnf_w, self.lnf_b)
        if targets is None:
            return ops.linear(h, self.wte)[..., :cfg.vocab_size]
        return ops.lm_head_xent(h, self.wte, targets, cfg.vocab_size)
