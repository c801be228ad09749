"""pdo-launch: the in-container launcher of a PaddleJob rank.

Reads the PaddleJob env contract (launch/env.py), derives the
torch.distributed contract, bootstraps RCCL (launch/bootstrap.py), reports
readiness, and runs the workload with periodic checkpoints and resume.
Replaces ``python -m paddle.distributed.launch train.py`` of the reference's
images (deploy/examples/resnet.yaml:14-19).

    python -m paddle_operator_amd.launch --workload gpt2 --model gpt2-medium --steps 100
    python -m paddle_operator_amd.launch --workload wide_deep --steps 200      # PS mode from env
    python -m paddle_operator_amd.launch --workload resnet50 --elastic         # elastic agent
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import time

T_START = time.time()


def parse_args(argv=None):
    ap = argparse.ArgumentParser(prog="pdo-launch")
    ap.add_argument("--workload", default="noop", choices=["gpt2", "resnet50", "wide_deep", "deepfm", "noop"])
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=0, help="untimed steps before the timed ones (--bench)")
    ap.add_argument("--bench", action="store_true",
                    help="benchmark protocol: --warmup untimed steps, then exactly --steps timed steps bracketed by "
                         "barrier + device synchronize; the record goes to pdo-kv /pdo/<job>/bench/<rank>")
    ap.add_argument("--batch", type=int, default=0, help="per-rank micro batch (0 = workload default)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--tiny", action="store_true", help="tiny model variant (CPU tests)")
    ap.add_argument("--backend", default=None, help="nccl (RCCL) | gloo; default by device")
    ap.add_argument("--nproc-per-pod", type=int, default=1)
    ap.add_argument("--ckpt-dir", default=os.environ.get("PDO_CKPT_DIR", ""))
    ap.add_argument("--ckpt-every", type=int, default=0)
    ap.add_argument("--ipc-probe", action="store_true", help="hipIpc handle exchange + xGMI copy probe")
    ap.add_argument("--elastic", action="store_true", help="force the elastic agent (default: from env)")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)  # elastic child
    ap.add_argument("--sync-ps", action="store_true")
    ap.add_argument("--log-every", type=int, default=10)
    ap.add_argument("--exit-after-ready", action="store_true")
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--throttle-ms", type=float, default=0.0, help=argparse.SUPPRESS)  # tests: stretch steps
    return ap.parse_args(argv)


def log(msg: str):
    print(f"[pdo-launch {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _install_sigterm(save_fn):
    def handler(signum, frame):
        try:
            save_fn()
        finally:
            os._exit(143)
    signal.signal(signal.SIGTERM, handler)


def run_collective(args, jenv) -> int:
    import torch
    import torch.distributed as dist

    from . import bootstrap
    from ..utils import checkpoint as ckpt
    from ..utils import trace

    if "RANK" not in os.environ or not args.worker:
        os.environ.update(jenv.torch_env(0, args.nproc_per_pod))
    b = bootstrap.init(T_START, backend=args.backend, timeout_s=args.timeout, ipc_probe=args.ipc_probe)
    dev = b.device
    trainer = None
    tokens_per_step = 0
    if args.workload == "gpt2":
        from ..models.gpt2 import GPT2Config
        from ..train import GPT2Trainer
        cfg = GPT2Config.named("gpt2-tiny" if args.tiny else args.model)
        seq = min(args.seq, cfg.n_positions)
        trainer = GPT2Trainer(cfg, args.batch or (2 if args.tiny else 32), seq, dev)
        trainer.sync_initial_weights()
        tokens_per_step = trainer.tokens_per_step()
    elif args.workload == "resnet50":
        from ..workloads.resnet import ResNetTrainer
        trainer = ResNetTrainer(args.batch or (4 if args.tiny else 256), dev, tiny=args.tiny)
        trainer.sync_initial_weights()
        tokens_per_step = trainer.B  # images
    start_step = 0
    if trainer is not None and args.ckpt_dir:
        st, start_step = ckpt.load_latest(args.ckpt_dir)
        if st is not None:
            if args.workload == "gpt2":
                trainer.flat.params.copy_(st["params"].to(dev))
                trainer.opt.load_state_dict({k: v.to(dev) if torch.is_tensor(v) else v
                                             for k, v in st["opt"].items()})
            else:
                trainer.load_state_dict(st)
            log(f"rank {b.rank}: resumed from step {start_step}")
    rec = bootstrap.report_ready(b, jenv.job_key(), jenv.kv_endpoints(),
                                 {"workload": args.workload, "resume_step": start_step})
    if args.exit_after_ready or trainer is None:
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()
        return 0

    if args.bench:
        return _bench(args, b, jenv, trainer, tokens_per_step, rec)

    def state():
        if args.workload == "gpt2":
            return {"params": trainer.flat.params, "opt": trainer.opt.state_dict()}
        return trainer.state_dict()

    step = start_step
    in_step = [False]
    if args.ckpt_dir and b.rank == 0:
        # a SIGTERM mid-step (arena half-updated) falls back to the last periodic checkpoint
        _install_sigterm(lambda: None if in_step[0] else ckpt.save(state(), args.ckpt_dir, step))
    t0 = time.perf_counter()
    last = t0
    done = 0
    while step < args.steps:
        in_step[0] = True
        with trace.range(f"step {step}"):
            loss = trainer.step()
        if args.throttle_ms:
            time.sleep(args.throttle_ms / 1e3)
        if dev.type == "cuda" and args.ckpt_dir:
            torch.cuda.current_stream(dev).synchronize()
        step += 1
        in_step[0] = False
        done += 1
        if args.ckpt_dir and args.ckpt_every and step % args.ckpt_every == 0 and b.rank == 0:
            with trace.range("checkpoint"):
                ckpt.save(state(), args.ckpt_dir, step)
        if step % args.log_every == 0 or step == args.steps:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            now = time.perf_counter()
            rate = tokens_per_step * b.world * args.log_every / max(now - last, 1e-9)
            last = now
            if b.rank == 0:
                log(f"step {step}/{args.steps} loss {float(loss.detach()):.4f} {rate:,.0f} "
                    f"{'tokens' if args.workload == 'gpt2' else 'img'}/s (job)")
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    if args.ckpt_dir and b.rank == 0:
        ckpt.save(state(), args.ckpt_dir, step)
    summary = {"rank": b.rank, "world": b.world, "steps": done, "seconds": dt,
               "throughput": tokens_per_step * b.world * done / max(dt, 1e-9), "final_step": step,
               "ready_s": rec["t_ready"] - T_START}
    print("PDO_DONE " + json.dumps(summary), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _bench(args, b, jenv, trainer, tokens_per_step, ready_rec) -> int:
    """The bench.py contract inside a launched rank: W untimed steps, then
    exactly K timed steps bracketed by barrier + device synchronize on both
    sides.  Every rank publishes its own elapsed time; the launcher parent
    (bench.py) takes the max over ranks."""
    import torch
    import torch.distributed as dist

    dev = b.device

    def fence():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        if dist.is_initialized():
            dist.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    loss = None
    for _ in range(args.warmup):
        loss = trainer.step()
    fence()
    t_wall0 = time.time()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step()
    fence()
    dt = time.perf_counter() - t0
    res = {"rank": b.rank, "world": b.world, "steps": args.steps, "warmup": args.warmup, "seconds": dt,
           "t_timed_start": t_wall0, "tokens_per_step_rank": tokens_per_step,
           "loss": float(loss.detach().float()) if loss is not None else None,
           "ready_s": ready_rec["t_ready"] - T_START, "t_ready": ready_rec["t_ready"],
           "backend": b.backend, "device": str(dev),
           "grad_reduce": getattr(getattr(trainer, "ddp", None), "grad_reduce", None),
           "buckets": len(trainer.flat.buckets) if hasattr(trainer, "flat") else None}
    if dev.type == "cuda":
        res["gpu_name"] = torch.cuda.get_device_name(dev)
        res["max_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 2**30, 2)
    if dist.is_initialized() and dist.get_world_size() > 1:
        res["comm"] = _comm_diag(trainer, fence, dev, dt / max(args.steps, 1))
    print("PDO_BENCH " + json.dumps(res), flush=True)
    kv = jenv.kv_endpoints()
    if kv:
        from ..kv.client import KVClient
        KVClient(kv).put(f"/pdo/{jenv.job_key()}/bench/{b.rank}", json.dumps(res))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


def _comm_diag(trainer, fence, dev, step_s, nosync_steps=3, iters=10):
    """Communication evidence for a multi-rank bench, measured AFTER the timed
    region (the bench record's timing is untouched):

    * ``exposed_ms``: timed step minus the same step with the gradient
      all-reduce switched off (``BucketedDDP.no_sync``) — the part of the
      bucketed RCCL traffic the backward did not hide;
    * ``allreduce_busbw_GBps``: one bucket-sized (64 MiB on GPU) bf16
      all-reduce, ring bus bandwidth = bytes · 2(n−1)/n / time — what xGMI
      delivers to this job's communicator.

    The no-sync steps leave the ranks' weights different; the job ends here."""
    import torch
    import torch.distributed as dist

    out = {}
    n = dist.get_world_size()
    ddp = getattr(trainer, "ddp", None)
    if ddp is not None and getattr(ddp, "enabled", False):
        with ddp.no_sync():
            trainer.step()
            fence()
            t0 = time.perf_counter()
            for _ in range(nosync_steps):
                trainer.step()
            fence()
        ns = (time.perf_counter() - t0) / nosync_steps
        out["step_ms"] = round(step_s * 1e3, 3)
        out["nosync_step_ms"] = round(ns * 1e3, 3)
        out["exposed_ms"] = round((step_s - ns) * 1e3, 3)
    nbytes = (64 << 20) if dev.type == "cuda" else (4 << 20)
    buf = torch.ones(nbytes // 2, dtype=torch.bfloat16, device=dev)
    for _ in range(3):
        dist.all_reduce(buf)
    fence()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(buf)
    fence()
    t = (time.perf_counter() - t0) / iters
    out["allreduce_bytes"] = nbytes
    out["allreduce_us"] = round(t * 1e6, 1)
    out["allreduce_busbw_GBps"] = round(nbytes * 2 * (n - 1) / n / t / 1e9, 1)
    return out


def run_ps(args, jenv) -> int:
    import datetime

    import torch
    import torch.distributed as dist
    import torch.distributed.rpc as rpc

    from . import bootstrap
    from ..models.wide_deep import WideDeepConfig, synthetic_batch
    from ..parallel import ps as psmod

    rank, world, master = jenv.ps_world()
    host, port = master.rsplit(":", 1)
    n_ps = len(jenv.pserver_endpoints)
    model = "deepfm" if args.workload == "deepfm" else "wide_deep"
    cfg = WideDeepConfig(vocab_per_slot=1000, model=model) if args.tiny else WideDeepConfig(model=model)
    n_heter = len(jenv.heter_endpoints)
    name = {"PSERVER": "ps", "HETER": "heter"}.get(jenv.role, "trainer") + str(jenv.trainer_id)
    opts = rpc.TensorPipeRpcBackendOptions(init_method=f"tcp://{host}:{int(port) + 1}", rpc_timeout=args.timeout,
                                           num_worker_threads=16)
    if jenv.role == "PSERVER":
        psmod.serve(jenv.trainer_id, n_ps, cfg)
    elif jenv.role == "HETER":
        psmod.serve_heter(cfg)  # dense tower on this worker's GPU (CPU without one)
    rpc.init_rpc(name, rank=rank, world_size=world, rpc_backend_options=opts)
    # gloo group on the reference's gloo HTTP endpoint (ps-0:2397) for barrier/metrics
    gloo = None
    if jenv.with_gloo and jenv.gloo_endpoint:
        gh, gp = jenv.gloo_endpoint.rsplit(":", 1)
        store = dist.TCPStore(gh, int(gp), world, is_master=(rank == 0), timeout=datetime.timedelta(seconds=120))
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world)
        gloo = True
    b = bootstrap.Bootstrapped(rank, world, 0, torch.device("cpu"), "rpc+gloo" if gloo else "rpc", T_START,
                               t_pg=time.time())
    bootstrap.report_ready(b, jenv.job_key(), jenv.kv_endpoints(), {"role": jenv.role, "workload": "wide_deep"})
    loss_sum = 0.0
    if jenv.role == "TRAINER" and not args.exit_after_ready:
        client = (psmod.HeterPSClient(n_ps, n_heter, cfg, sync=args.sync_ps, first=jenv.trainer_id) if n_heter
                  else psmod.PSClient(n_ps, cfg, sync=args.sync_ps))
        gen = torch.Generator().manual_seed(1000 + jenv.trainer_id)
        B = args.batch or 512
        t0 = time.perf_counter()
        losses = []
        for step in range(args.steps):
            ids, dense, label = synthetic_batch(cfg, B, gen)
            losses.append(client.step(ids, dense, label))
            if (step + 1) % args.log_every == 0:
                log(f"trainer{jenv.trainer_id} step {step + 1} loss {sum(losses[-args.log_every:]) / args.log_every:.4f}")
        client.flush()
        dt = time.perf_counter() - t0
        loss_sum = sum(losses[-10:]) / max(1, len(losses[-10:]))
        print("PDO_DONE " + json.dumps({"role": "TRAINER", "trainer": jenv.trainer_id, "steps": args.steps,
                                        "seconds": dt, "samples_per_s": B * args.steps / dt,
                                        "first_loss": losses[0] if losses else None, "last_loss": loss_sum,
                                        "server_stats": client.server_stats(),
                                        "heter_stats": client.heter_stats() if n_heter else None}), flush=True)
    if gloo:
        t = torch.tensor([loss_sum])
        dist.all_reduce(t)
        dist.destroy_process_group()
    rpc.shutdown()  # blocks until every worker is done (pservers wait here)
    return 0


def main(argv=None) -> int:
    args = parse_args(argv)
    from .env import JobEnv
    jenv = JobEnv.from_env()
    jenv.check_supported()
    log(f"role={jenv.role} id={jenv.trainer_id} mode={jenv.mode} elastic={jenv.elastic} workload={args.workload}")
    hang_dump = float(os.environ.get("PDO_HANG_DUMP_S", "0") or 0)
    if hang_dump > 0:
        # hang diagnostics: every thread's Python stack to the pod log every N s
        # (a rank stuck in a collective shows where; no debugger attached)
        import faulthandler
        faulthandler.dump_traceback_later(hang_dump, repeat=True, file=sys.stderr)
    if jenv.mode == "PS" or args.workload in ("wide_deep", "deepfm") and jenv.pserver_endpoints:
        return run_ps(args, jenv)
    if (jenv.elastic or args.elastic) and not args.worker:
        from .elastic import run_agent
        return run_agent(args, jenv, argv if argv is not None else sys.argv[1:])
    return run_collective(args, jenv)


if __name__ == "__main__":
    sys.exit(main())
