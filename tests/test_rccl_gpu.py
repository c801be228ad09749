"""RCCL on the hardware: communicator, DDP buckets, IPC bootstrap (1×MI355X).

Every GPU process group here is backend ``nccl`` — on ROCm that IS RCCL:

* the launcher bootstrap (launch/bootstrap.py) builds the RCCL communicator
  eagerly (``device_id``) even for a 1-rank job and runs the warm-up
  all-reduce, so "ready" includes comm init;
* ``BucketedDDP(enabled=True)`` over RCCL at world 1 on the HIP training path:
  every bucket all-reduce runs (identity at world 1), gradients must be
  unchanged bit for bit, in both reduction precisions (bf16 wire / fp32
  staging through csrc/hip/bucket.hip);
* hipIpc: two processes on the same GPU exchange a device buffer through
  ``hipIpcGetMemHandle`` / ``hipIpcOpenMemHandle`` (the launcher's intra-node
  bootstrap primitive) — read and write across the process boundary;
* ``bin/pdo-allreduce-bench`` (C++ RCCL sweep) runs and reports JSON lines.
"""
import json
import os
import subprocess

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def rccl_world1(cuda):
    assert not dist.is_initialized()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=cuda)
    yield cuda
    dist.destroy_process_group()


def _cfg():
    from paddle_operator_amd.models.gpt2 import GPT2Config
    return GPT2Config(vocab_size=1000, n_positions=256, n_embd=256, n_layer=2, n_head=4)


def _grads(dev, ddp_mode):
    """Arena gradients of one step; ddp_mode None = no DDP, else RCCL buckets in that precision."""
    from paddle_operator_amd.models.gpt2 import GPT2
    from paddle_operator_amd.parallel.ddp import BucketedDDP
    from paddle_operator_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    cfg = _cfg()
    model = GPT2(cfg).to(device=dev, dtype=torch.bfloat16)
    flat = FlatParams(model, dtype=torch.bfloat16, device=dev, bucket_bytes=256 << 10, late=("wte",))
    ddp = BucketedDDP(flat, enabled=ddp_mode is not None, grad_reduce=ddp_mode)
    if ddp_mode is not None:
        assert len(flat.buckets) > 4
        ddp.broadcast_params(0)
    g = torch.Generator().manual_seed(3)
    idx = torch.randint(0, cfg.vocab_size, (4, 129), generator=g).to(dev)
    for _ in range(2):
        flat.zero_grad()
        ddp.prepare()
        model(idx[:, :-1], idx[:, 1:]).backward()
        ddp.finish()
    torch.cuda.synchronize()
    if ddp_mode is not None:
        assert all(ddp._launched), "every bucket all-reduce must have been issued"
        assert ddp.grad_scale == 1.0
    return flat.grads.clone()


def test_bucketed_ddp_over_rccl_world1(rccl_world1):
    os.environ["PDO_OPS"] = "hip"
    assert dist.get_backend() == "nccl"
    ref = _grads(rccl_world1, None)
    for mode in ("bf16", "fp32"):
        got = _grads(rccl_world1, mode)
        assert torch.equal(got, ref), f"{mode}: RCCL bucket reduction changed the gradients at world 1"


def test_bucket_kernels_flatten_unflatten_cast(cuda):
    from paddle_operator_amd import _native
    m = _native.require_hip()
    for dt in (torch.bfloat16, torch.float32):
        ts = [torch.randn(n, device=cuda).to(dt) for n in (5, 1000, 3, 4096)]
        offs, o = [], 0
        for t in ts:
            offs.append(o)
            o += t.numel() + 7  # padding between tensors stays untouched
        flat = torch.full((o,), 9.0, device=cuda, dtype=dt)
        m.flatten_scale(ts, flat, offs, 0.5, False)
        for t, off in zip(ts, offs):
            torch.testing.assert_close(flat[off:off + t.numel()].float(), (t.float() * 0.5).to(dt).float())
            assert float(flat[off + t.numel()]) == 9.0
        outs = [torch.zeros_like(t) for t in ts]
        m.flatten_scale(outs, flat, offs, 1.0, True)
        for t, u in zip(ts, outs):
            torch.testing.assert_close(u.float(), (t.float() * 0.5).to(dt).float())
    g = torch.randn(8192, device=cuda).to(torch.bfloat16)
    st = torch.empty(8192, device=cuda)
    m.cast_scale_bf16_f32(g, st, 0.125)
    torch.testing.assert_close(st, g.float() * 0.125, rtol=0, atol=0)
    back = torch.empty_like(g)
    m.cast_f32_bf16(st * 8, back)
    assert torch.equal(back, g)


def test_bootstrap_builds_rccl_at_world1(cuda, monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    from paddle_operator_amd.launch import bootstrap
    import time
    b = bootstrap.init(time.time())
    try:
        assert dist.is_initialized() and dist.get_backend() == "nccl" and b.backend == "nccl"
        assert b.t_pg >= b.t_start
        t = torch.full((4,), 3.0, device=cuda)
        dist.all_reduce(t)
        assert float(t.sum()) == 12.0
    finally:
        dist.destroy_process_group()


def _ipc_owner(handle_q, written_q, result_q):
    torch.cuda.set_device(0)
    from paddle_operator_amd import _native
    m = _native.require_hip()
    # a sub-allocation: the tensor does not start at its allocation base
    pool = torch.zeros(3 << 20, dtype=torch.uint8, device="cuda")
    buf = pool[1 << 20: 2 << 20]
    buf.fill_(77)
    torch.cuda.synchronize()
    h, off = m.ipc_get_handle(buf)
    handle_q.put((h, off, buf.numel()))
    assert written_q.get(timeout=120) == "written"
    torch.cuda.synchronize()
    ok = bool((buf[:4096] == 5).all()) and bool((buf[4096:] == 77).all()) and bool((pool[:1 << 20] == 0).all())
    result_q.put("ok" if ok else "bad")


def _ipc_peer(handle_q, written_q):
    torch.cuda.set_device(0)
    from paddle_operator_amd import _native
    m = _native.require_hip()
    h, off, n = handle_q.get(timeout=120)
    peer = m.ipc_open_handle(h, n, 0, off)
    got = peer.clone()
    torch.cuda.synchronize()
    assert bool((got == 77).all()), "peer read the wrong bytes"
    peer[:4096].fill_(5)
    torch.cuda.synchronize()
    del peer
    written_q.put("written")


def test_hip_ipc_cross_process_same_gpu(cuda):
    """Owner exports a sub-allocated buffer; a second process maps it, reads it and writes into it."""
    ctx = mp.get_context("spawn")
    handle_q, written_q, result_q = ctx.Queue(), ctx.Queue(), ctx.Queue()
    pa = ctx.Process(target=_ipc_owner, args=(handle_q, written_q, result_q))
    pb = ctx.Process(target=_ipc_peer, args=(handle_q, written_q))
    pa.start()
    pb.start()
    pb.join(180)
    pa.join(180)
    assert pb.exitcode == 0 and pa.exitcode == 0, (pa.exitcode, pb.exitcode)
    assert result_q.get(timeout=10) == "ok"


def test_allreduce_bench_binary_runs(cuda):
    exe = os.path.join(REPO, "bin", "pdo-allreduce-bench")
    assert os.path.exists(exe), "build first (tools/build.py)"
    r = subprocess.run([exe, "--gpus", "1", "--min", "1M", "--max", "16M", "--iters", "5", "--warmup", "2"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(rows) >= 5 and all(x["ranks"] == 1 and x["us"] > 0 for x in rows if "us" in x), r.stdout


def test_warm_slot_ready_on_gpu(cuda):
    """bench.py --ready-only through the operator with the node's GPU-warm slot:
    every rank is served by a slot (HIP + RCCL code already loaded) and the
    job's own communicator init is no longer dominated by RCCL kernel loading
    (≈1.1 s cold, profiles/r2_launched_bench_1gpu.md)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--ready-only", "--ready-trials", "3"],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    ready = rec["ready"]
    assert ready["warm_slot_fraction"] == 1.0, ready
    assert ready["rank_phases_p50"]["comm"] < 0.5, ready
    assert ready["p50"] < 1.0, ready
