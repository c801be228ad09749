"""Parameter-server training over torch.distributed.rpc (TensorPipe / TCP).

PaddleJob ``Mode=PS`` (reference: controllers/paddlejob_helper.go:191-199,
role env TRAINING_ROLE=PSERVER/TRAINER, PADDLE_PSERVERS_IP_PORT_LIST; the
Paddle image runs brpc-based PS on CPU, deploy/examples/wide_and_deep.yaml).

* Each pserver owns a contiguous row shard of the sparse tables (deep
  embeddings + wide weights) and updates it with row-wise Adagrad; pserver 0
  also owns the dense tower (Adam).
* A trainer step pulls only the rows its batch touches (one RPC per shard,
  issued concurrently), runs forward/backward locally, and pushes the row
  gradients (+ dense grads to pserver 0) asynchronously (async SGD, the
  Paddle PS default for CTR models); ``sync=True`` waits for the pushes.
* RPC world: pservers are ranks 0..P-1 ("ps{i}"), trainers P.. ("trainer{j}");
  the TensorPipe store listens on pserver 0's PADDLE_PORT+1.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional

import torch
import torch.distributed.rpc as rpc

from ..models.wide_deep import WideDeepConfig, make_tower, shard_rows

_SERVER: Optional["ShardServer"] = None


class ShardServer:
    def __init__(self, shard: int, lo: int, hi: int, cfg: WideDeepConfig, lr: float = 0.05,
                 dense_lr: float = 1e-3, seed: int = 0):
        g = torch.Generator().manual_seed(seed + shard)
        self.shard, self.lo, self.hi, self.cfg = shard, lo, hi, cfg
        n = hi - lo
        self.deep = torch.randn(n, cfg.emb_dim, generator=g) * 0.01
        self.wide = torch.zeros(n, 1)
        self.deep_acc = torch.full((n, cfg.emb_dim), 0.1)
        self.wide_acc = torch.full((n, 1), 0.1)
        self.lr = lr
        self.lock = threading.Lock()
        self.pushes = 0
        self.tower: Optional[DeepTower] = None
        if shard == 0:
            torch.manual_seed(seed)
            self.tower = make_tower(cfg)
            self.opt = torch.optim.Adam(self.tower.parameters(), lr=dense_lr)

    def pull(self, ids: torch.Tensor):
        local = ids - self.lo
        with self.lock:
            return self.deep[local].clone(), self.wide[local].clone()

    def push(self, ids: torch.Tensor, g_deep: torch.Tensor, g_wide: torch.Tensor):
        local = ids - self.lo
        with self.lock:
            # row-wise Adagrad (duplicates pre-summed by the trainer)
            self.deep_acc.index_add_(0, local, g_deep * g_deep)
            self.wide_acc.index_add_(0, local, g_wide * g_wide)
            self.deep.index_add_(0, local, -self.lr * g_deep / self.deep_acc[local].sqrt())
            self.wide.index_add_(0, local, -self.lr * g_wide / self.wide_acc[local].sqrt())
            self.pushes += 1
        return True

    def pull_dense(self) -> Dict[str, torch.Tensor]:
        with self.lock:
            return {k: v.detach().clone() for k, v in self.tower.state_dict().items()}

    def push_dense(self, grads: Dict[str, torch.Tensor]):
        with self.lock:
            for n, p in self.tower.named_parameters():
                p.grad = grads[n]
            self.opt.step()
            self.opt.zero_grad(set_to_none=True)
        return True

    def stats(self):
        return {"shard": self.shard, "rows": self.hi - self.lo, "pushes": self.pushes}


# ---- RPC entry points (executed on the pserver) ----------------------------
def _pull(ids):
    return _SERVER.pull(ids)


def _push(ids, gd, gw):
    return _SERVER.push(ids, gd, gw)


def _pull_dense():
    return _SERVER.pull_dense()


def _push_dense(grads):
    return _SERVER.push_dense(grads)


def _stats():
    return _SERVER.stats()


def serve(shard: int, n_ps: int, cfg: WideDeepConfig, **kw):
    """Install this process's shard (call after rpc.init_rpc)."""
    global _SERVER
    lo, hi = shard_rows(cfg.rows, n_ps)[shard]
    _SERVER = ShardServer(shard, lo, hi, cfg, **kw)
    return _SERVER


class PSClient:
    """Trainer side of the PS protocol."""

    def __init__(self, n_ps: int, cfg: WideDeepConfig, sync: bool = False):
        self.n_ps = n_ps
        self.cfg = cfg
        self.sync = sync
        self.bounds = shard_rows(cfg.rows, n_ps)
        self.tower = make_tower(cfg)
        self._pending: List = []

    def _split(self, uniq: torch.Tensor):
        out = []
        for lo, hi in self.bounds:
            m = (uniq >= lo) & (uniq < hi)
            out.append(uniq[m])
        return out

    def step(self, ids: torch.Tensor, dense: torch.Tensor, label: torch.Tensor) -> float:
        uniq, inv = torch.unique(ids, return_inverse=True)
        parts = self._split(uniq)
        futs = [rpc.rpc_async(f"ps{i}", _pull, args=(p,)) if p.numel() else None for i, p in enumerate(parts)]
        dense_fut = rpc.rpc_async("ps0", _pull_dense)
        # wait for the previous step's pushes before using fresh rows (bounded staleness = 1)
        for f in self._pending:
            f.wait()
        self._pending = []
        rows_d, rows_w = [], []
        for f, p in zip(futs, parts):
            if f is None:
                continue
            d, w = f.wait()
            rows_d.append(d)
            rows_w.append(w)
        deep_rows = torch.cat(rows_d).requires_grad_()
        wide_rows = torch.cat(rows_w).requires_grad_()
        self.tower.load_state_dict(dense_fut.wait())
        self.tower.zero_grad(set_to_none=True)
        # rows were gathered in shard order == sorted order of uniq → index by inverse map
        logit = self.tower(deep_rows[inv], wide_rows[inv], dense)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, label)
        loss.backward()
        off = 0
        for i, p in enumerate(parts):
            n = p.numel()
            if not n:
                continue
            self._pending.append(rpc.rpc_async(f"ps{i}", _push, args=(p, deep_rows.grad[off:off + n].clone(),
                                                                      wide_rows.grad[off:off + n].clone())))
            off += n
        grads = {n: p.grad.detach().clone() for n, p in self.tower.named_parameters()}
        self._pending.append(rpc.rpc_async("ps0", _push_dense, args=(grads,)))
        if self.sync:
            for f in self._pending:
                f.wait()
            self._pending = []
        return float(loss.detach())

    def flush(self):
        for f in self._pending:
            f.wait()
        self._pending = []

    def server_stats(self):
        return [rpc.rpc_sync(f"ps{i}", _stats) for i in range(self.n_ps)]


# ---------------------------------------------------------------------------
# Heterogeneous PS (PaddleJob ``spec.heter``; role HETER, PADDLE_HETER_ENDPOINTS,
# reference paddlejob_types.go:40,47,146-147 / paddlejob_helper.go:266-268):
# CPU trainers keep the sparse side (pull rows from the pservers, push row
# gradients), GPU heter workers own the dense tower and run its forward /
# backward / Adam on an MI355X.  RPC names "heter{i}", ranks after the trainers.
# ---------------------------------------------------------------------------
_HETER: Optional["HeterServer"] = None


class HeterServer:
    def __init__(self, cfg: WideDeepConfig, device=None, lr: float = 1e-3, seed: int = 0):
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        torch.manual_seed(seed)
        self.tower = make_tower(cfg).to(self.device)
        self.opt = torch.optim.Adam(self.tower.parameters(), lr=lr)
        self.lock = threading.Lock()
        self.steps = 0

    def step(self, deep_rows, wide_rows, inv, dense, label):
        d = self.device
        with self.lock:
            dr = deep_rows.to(d, non_blocking=True).requires_grad_()
            wr = wide_rows.to(d, non_blocking=True).requires_grad_()
            logit = self.tower(dr[inv.to(d)], wr[inv.to(d)], dense.to(d))
            loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, label.to(d))
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            self.opt.step()
            self.steps += 1
            return float(loss.detach()), dr.grad.cpu(), wr.grad.cpu()

    def stats(self):
        return {"heter_steps": self.steps, "device": str(self.device)}


def _heter_step(deep_rows, wide_rows, inv, dense, label):
    return _HETER.step(deep_rows, wide_rows, inv, dense, label)


def _heter_stats():
    return _HETER.stats()


def serve_heter(cfg: WideDeepConfig, device=None, **kw):
    global _HETER
    _HETER = HeterServer(cfg, device, **kw)
    return _HETER


class HeterPSClient(PSClient):
    """Trainer that offloads the dense tower to heter workers (round robin)."""

    def __init__(self, n_ps: int, n_heter: int, cfg: WideDeepConfig, sync: bool = False, first: int = 0):
        super().__init__(n_ps, cfg, sync)
        self.n_heter = n_heter
        self._rr = first

    def step(self, ids, dense, label) -> float:
        uniq, inv = torch.unique(ids, return_inverse=True)
        parts = self._split(uniq)
        futs = [rpc.rpc_async(f"ps{i}", _pull, args=(p,)) if p.numel() else None for i, p in enumerate(parts)]
        for f in self._pending:
            f.wait()
        self._pending = []
        rows_d, rows_w = [], []
        for f in futs:
            if f is None:
                continue
            d, w = f.wait()
            rows_d.append(d)
            rows_w.append(w)
        h = self._rr % self.n_heter
        self._rr += 1
        loss, gd, gw = rpc.rpc_sync(f"heter{h}", _heter_step,
                                    args=(torch.cat(rows_d), torch.cat(rows_w), inv, dense, label))
        off = 0
        for i, p in enumerate(parts):
            n = p.numel()
            if not n:
                continue
            self._pending.append(rpc.rpc_async(f"ps{i}", _push, args=(p, gd[off:off + n], gw[off:off + n])))
            off += n
        if self.sync:
            self.flush()
        return loss

    def heter_stats(self):
        return [rpc.rpc_sync(f"heter{i}", _heter_stats) for i in range(self.n_heter)]
