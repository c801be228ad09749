"""Wide & Deep CTR model (BASELINE config 1: PS-mode PaddleJob, 1 pserver + 1
trainer on CPU — the reference's deploy/examples/wide_and_deep.yaml).

Criteo-like synthetic input: 26 categorical slots (hashed into per-slot
vocabularies) + 13 dense features.  Wide part: per-feature scalar weights
(an embedding of dim 1); deep part: 16-d embeddings → MLP(400, 400, 400).

For parameter-server training the embedding tables are *sharded by row*
across pservers (``shard_rows``) and trainers exchange only the rows of their
batch (parallel/ps.py); the dense MLP lives on pserver 0.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn


@dataclass
class WideDeepConfig:
    n_sparse: int = 26
    vocab_per_slot: int = 10000
    emb_dim: int = 16
    n_dense: int = 13
    hidden: tuple = (400, 400, 400)
    model: str = "wide_deep"  # "wide_deep" | "deepfm" (deploy/examples/deepfm.yaml)

    @property
    def rows(self) -> int:
        return self.n_sparse * self.vocab_per_slot


class DeepTower(nn.Module):
    """Dense part (MLP over [embeddings, dense features])."""

    def __init__(self, cfg: WideDeepConfig):
        super().__init__()
        dims = [cfg.n_sparse * cfg.emb_dim + cfg.n_dense] + list(cfg.hidden)
        layers = []
        for a, b in zip(dims[:-1], dims[1:]):
            layers += [nn.Linear(a, b), nn.ReLU()]
        layers.append(nn.Linear(dims[-1], 1))
        self.mlp = nn.Sequential(*layers)
        self.wide_bias = nn.Parameter(torch.zeros(1))

    def forward(self, deep_emb, wide_w, dense):
        # deep_emb [B, S, D], wide_w [B, S, 1], dense [B, n_dense]
        x = torch.cat([deep_emb.flatten(1), dense], dim=1)
        return self.mlp(x).squeeze(1) + wide_w.sum(dim=(1, 2)) + self.wide_bias


class DeepFMTower(DeepTower):
    """DeepFM: the wide (first-order) term + a factorisation-machine
    second-order term over the slot embeddings + the deep MLP, all sharing the
    same sparse tables (so the PS protocol is unchanged)."""

    def forward(self, deep_emb, wide_w, dense):
        s = deep_emb.sum(dim=1)  # [B, D]
        fm = 0.5 * (s * s - (deep_emb * deep_emb).sum(dim=1)).sum(dim=1)
        return super().forward(deep_emb, wide_w, dense) + fm


def make_tower(cfg: WideDeepConfig) -> DeepTower:
    return DeepFMTower(cfg) if cfg.model == "deepfm" else DeepTower(cfg)


class WideDeep(nn.Module):
    """Single-process model (Single / Collective modes and tests)."""

    def __init__(self, cfg: WideDeepConfig = WideDeepConfig()):
        super().__init__()
        self.cfg = cfg
        self.deep_emb = nn.Embedding(cfg.rows, cfg.emb_dim)
        self.wide = nn.Embedding(cfg.rows, 1)
        nn.init.normal_(self.deep_emb.weight, std=0.01)
        nn.init.zeros_(self.wide.weight)
        self.tower = make_tower(cfg)

    def forward(self, ids, dense):
        return self.tower(self.deep_emb(ids), self.wide(ids), dense)


def synthetic_batch(cfg: WideDeepConfig, batch: int, gen: torch.Generator, device="cpu"):
    """Global row ids (slot offset + hashed id), dense features, click labels.

    Labels come from a fixed random linear rule on the features so the model
    has something learnable (loss falls) while the data stays synthetic.
    """
    slot_ids = torch.randint(0, cfg.vocab_per_slot, (batch, cfg.n_sparse), generator=gen)
    ids = slot_ids + torch.arange(cfg.n_sparse) * cfg.vocab_per_slot
    dense = torch.rand(batch, cfg.n_dense, generator=gen)
    score = (slot_ids % 7 == 0).float().mean(1) * 4 + dense[:, 0] - 1.0
    label = (score + 0.1 * torch.randn(batch, generator=gen) > 0).float()
    return ids.to(device), dense.to(device), label.to(device)


def shard_rows(rows: int, n_shards: int):
    """Contiguous row ranges per pserver: [(lo, hi), ...]."""
    per = (rows + n_shards - 1) // n_shards
    return [(i * per, min(rows, (i + 1) * per)) for i in range(n_shards)]
