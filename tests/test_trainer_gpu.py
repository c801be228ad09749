"""The GPT-2 production trainer anchored to fp32.

``GPT2Trainer.step()`` exactly as bench.py runs it — split tied-embedding
gradient slot, batched Wᵀ operands (``enable_wt``), deferred bias / norm column
sums, ``BucketedDDP.finish(opt)`` with per-bucket global-norm partials (DDP on:
a 1-rank RCCL communicator with ``PDO_DDP_ALWAYS=1``, so the hooks, bucket
launches and partials all run), clipped fused ``FlatAdamW`` over the bf16
arena with fp32 master weights — at GPT-2-medium width (C = 1024, 16 heads,
vocab 50304, S = 1024, B = 8, 2 layers) for 3 steps.

Teacher-forced per step (the trajectories of a sign-like Adam update diverge
chaotically after one step: a single near-zero gradient whose bf16 sign differs
moves one element by 2·lr, 6 % of a 1024-element update — measured, round 6):

* gradients: at the trainer's own weights of that step, the production
  gradient (arena, after the split fold) against the SAME weights in fp32 with
  plain torch ops (``PDO_OPS=torch``) — every parameter within 1.5× the
  framework's own bf16 error at those weights (+ 0.005) — and the loss;
* optimizer: the fused clipped AdamW's master-weight update against
  ``torch.optim.AdamW``'s formula + ``clip_grad_norm_`` in fp32 (fp64 norm)
  applied to the same gradients and the trainer's own moments;
* the global-norm partials computed per bucket during the drain equal a
  one-pass recomputation bit for bit (ddp.py:139).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STEPS = 3
B, S = 8, 1024


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-30))


def _worker(port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PDO_OPS="hip", PDO_DDP_ALWAYS="1")
    import torch.distributed as dist

    from paddle_operator_amd.models.gpt2 import GPT2, GPT2Config
    from paddle_operator_amd.train import GPT2Trainer

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=dev)
    cfg = GPT2Config(n_embd=1024, n_layer=2, n_head=16)
    tr = GPT2Trainer(cfg, B, S, dev, bucket_mb=16)  # ≈ 10 buckets: partials and launches per bucket
    tr.sync_initial_weights()
    assert tr.ddp.enabled and len(tr.flat.buckets) >= 2 and tr.flat.aux_slots, "production composition not active"
    opt, flat = tr.opt, tr.flat
    slots = flat.slots
    view = lambda buf, s: buf[s.offset:s.offset + s.numel].view(s.shape)  # noqa: E731
    with torch.device(dev):
        ref = GPT2(cfg)  # fp32
        fw = GPT2(cfg).bfloat16()  # the framework in bf16

    def ref_grads(model, master, x, y):
        """Loss and gradients of ``model`` (torch ops) at the trainer's master weights."""
        params = dict(model.named_parameters())
        with torch.no_grad():
            for s in slots:
                params[s.name].copy_(view(master, s))
        model.zero_grad(set_to_none=True)
        os.environ["PDO_OPS"] = "torch"
        try:
            loss = model(x, y)
            loss.backward()
        finally:
            os.environ["PDO_OPS"] = "hip"
        return float(loss.item()), {n: p.grad.float() for n, p in params.items()}

    res = {"loss": [], "norm_bits_equal": [], "grad_errs": [], "opt_err": [], "clip": []}
    for k in range(STEPS):
        x, y = tr.batch()
        master0, m0, v0 = opt.master.clone(), opt.m.clone(), opt.v.clone()
        loss_h = float(tr.step(x, y).item())
        # the drain's per-bucket partials (already summed into _norm_buf) vs a fresh one-pass sum
        drained = opt._norm_buf[0].clone()
        fresh = opt.grad_norm_sq(tr.ddp.grad_scale).clone()
        res["norm_bits_equal"].append(bool(torch.equal(drained, fresh)))
        g_h = {s.name: view(flat.param_grads, s).float() * tr.ddp.grad_scale for s in slots}
        loss_r, g_r = ref_grads(ref, master0, x, y)
        loss_f, g_f = ref_grads(fw, master0, x, y)
        res["loss"].append((loss_h, loss_r, loss_f))
        res["grad_errs"].append({n: (_rel(g_h[n], g_r[n]), _rel(g_f[n], g_r[n])) for n in g_h})
        # optimizer: torch's AdamW formula + clip on the trainer's own gradients and moments
        gflat = flat.param_grads.float() * tr.ddp.grad_scale
        norm = float(gflat.double().norm())
        c = min(1.0, opt.max_grad_norm / (norm + 1e-6))
        res["clip"].append((norm, float(drained.sqrt()), c))
        g = gflat * c
        t = opt.step_count
        bc1, bc2 = 1 - opt.b1 ** t, 1 - opt.b2 ** t
        m1 = opt.b1 * m0 + (1 - opt.b1) * g
        v1 = opt.b2 * v0 + (1 - opt.b2) * g * g
        dec = flat.decay_chunks.repeat_interleave(flat.numel // flat.decay_chunks.numel())
        want = master0 * (1 - opt.lr * opt.wd * dec) - opt.lr * (m1 / bc1) / ((v1 / bc2).sqrt() + opt.eps)
        res["opt_err"].append({s.name: _rel(view(opt.master, s) - view(master0, s), view(want, s) - view(master0, s))
                               for s in slots})
    torch.cuda.synchronize()
    dist.destroy_process_group()
    torch.save(res, out)


def test_gpt2_trainer_steps_vs_fp32(tmp_path, cuda):
    out = str(tmp_path / "anchor.pt")
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_worker, args=(_port(), out))
    p.start()
    p.join(600)
    assert p.exitcode == 0, p.exitcode
    res = torch.load(out, weights_only=True)
    d = os.environ.get("PDO_TEST_DUMP_DIR")
    if d:  # evidence for profiles/: per step losses, norm check, per-parameter (hip, framework bf16) errors
        import json
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "gpt2_trainer_anchor.json"), "w") as f:
            json.dump({k: v for k, v in res.items()}, f, indent=0)
    assert all(res["norm_bits_equal"]), res["norm_bits_equal"]
    for k in range(STEPS):
        lh, lr_, lf = res["loss"][k]
        assert abs(lh - lr_) < 1e-2, (k, lh, lr_, lf)
        norm, drained, _ = res["clip"][k]
        assert abs(norm - drained) < 1e-4 * norm, (k, norm, drained)  # the drained partials' norm is the norm
        bad = {n: (round(eh, 4), round(ef, 4)) for n, (eh, ef) in res["grad_errs"][k].items()
               if not eh <= 1.5 * ef + 0.005}
        assert not bad, ("gradients", k, bad)
        bad = {n: e for n, e in res["opt_err"][k].items() if not e < 1e-4}
        assert not bad, ("optimizer update", k, bad)
