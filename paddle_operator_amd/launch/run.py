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
    ap.add_argument("--no-graph", dest="graph", action="store_false",
                    help="resnet50: keep the step eager (default on one GPU rank: captured once into a HIP graph "
                         "and replayed, workloads/resnet.py; multi-rank steps stay eager)")
    ap.add_argument("--backend", default=None, help="nccl (RCCL) | gloo; default by device")
    ap.add_argument("--nproc-per-pod", type=int, default=int(os.environ.get("PDO_NPROC_PER_POD", "1") or 1),
                    help="ranks this pod runs, one per GPU it was given (amd.com/gpu: N): RANK = "
                         "PADDLE_TRAINER_ID·N + local, WORLD_SIZE = PADDLE_TRAINERS_NUM·N.  One pod with all of a "
                         "node's GPUs is the xGMI layout: RCCL sees every peer GPU in one IPC namespace")
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

    if os.environ.get("PDO_LOCAL_CHILD") != "1" and ("RANK" not in os.environ or not args.worker):
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
        trainer = ResNetTrainer(args.batch or (4 if args.tiny else 256), dev, tiny=args.tiny, graph=args.graph)
        trainer.sync_initial_weights()
        tokens_per_step = trainer.B  # images
    start_step = 0
    if trainer is not None and args.ckpt_dir:
        st, start_step = ckpt.load_latest(args.ckpt_dir)
        if st is not None:
            if args.workload == "gpt2":
                trainer.flat.load_params(st["params"])
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
           "buckets": len(trainer.flat.buckets) if hasattr(trainer, "flat") else None,
           "hip_graph": getattr(trainer, "_graph", None) is not None}
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
    * ``buckets``: the job's bucket count and sizes (bytes);
    * ``allreduce_sweep``: bf16 all-reduce busbw at 4 … 256 MiB (1 … 8 MiB on
      CPU) — the knee ``utils/topology.py bucket_bytes_for`` is tuned from
      (``knee_bytes``: the smallest size within 90 % of the best busbw);
      ``allreduce_busbw_GBps`` keeps the 64 MiB point;
    * ``ipc_gbps``: hipIpc handle exchange + a 64 MiB peer copy per same-node
      pair (the xGMI link the bootstrap probe sees), GPU only.

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
    flat = getattr(trainer, "flat", None)
    if flat is not None and getattr(flat, "buckets", None):
        esz = flat.params.element_size()
        out["buckets"] = {"count": len(flat.buckets), "bytes": [int(bk.numel * esz) for bk in flat.buckets],
                          # split tied weights: their head-gradient slot is bucket 0
                          "split": [a.name for a in getattr(flat, "aux_slots", [])],
                          "first": [s.name for s in flat.buckets[0].slots][:4]}
    sizes_mib = (4, 8, 16, 32, 64, 128, 256) if dev.type == "cuda" else (1, 2, 4, 8)
    buf = torch.ones((max(sizes_mib) << 20) // 2, dtype=torch.bfloat16, device=dev)
    sweep = []
    for mib in sizes_mib:
        view = buf[: (mib << 20) // 2]
        reps = iters if mib <= 64 else max(3, iters // 2)
        for _ in range(2):
            dist.all_reduce(view)
        fence()
        t0 = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(view)
        fence()
        t = (time.perf_counter() - t0) / reps
        sweep.append({"bytes": mib << 20, "us": round(t * 1e6, 1),
                      "busbw_GBps": round((mib << 20) * 2 * (n - 1) / n / t / 1e9, 1)})
    del buf
    out["allreduce_sweep"] = sweep
    best = max(p["busbw_GBps"] for p in sweep)
    out["knee_bytes"] = next(p["bytes"] for p in sweep if p["busbw_GBps"] >= 0.9 * best)
    ref = next((p for p in sweep if p["bytes"] == 64 << 20), sweep[-1])
    out["allreduce_bytes"] = ref["bytes"]
    out["allreduce_us"] = ref["us"]
    out["allreduce_busbw_GBps"] = ref["busbw_GBps"]
    if dev.type == "cuda":
        try:
            from .bootstrap import ipc_probe_run
            out["ipc_gbps"] = ipc_probe_run(dev)
        except Exception as e:  # diagnostics never fail the bench
            out["ipc_gbps"] = f"unavailable: {e}"
    return out


def spawn_local(args, jenv, argv) -> int:
    """--nproc-per-pod N: the pod's entry process becomes a supervisor of N
    local ranks, forked before anything in this process touches HIP.  Local
    rank i gets RANK = PADDLE_TRAINER_ID·N + i, LOCAL_RANK = i and device i of
    the pod's GPUs (HIP_VISIBLE_DEVICES under a device plugin, or PDO_GPU_IDS
    when the agent exposes every GPU — launch/bootstrap.py picks it), so all N
    devices stay visible to every rank and RCCL connects them peer to peer over
    xGMI.  SIGTERM/SIGINT are forwarded; the first rank to fail takes the
    others down (torchrun's behaviour) and its status is the pod's.
    Replaces what ``paddle.distributed.launch`` does per pod in the reference's
    images (deploy/examples/resnet.yaml:14-19)."""
    import signal
    if "torch" in sys.modules:
        import torch
        if torch.cuda.is_initialized():  # forking a HIP-initialised process is not allowed
            raise RuntimeError("--nproc-per-pod: HIP already initialised in the pod's entry process")
    n = args.nproc_per_pod
    gpus = os.environ.get("PDO_GPU_IDS") or os.environ.get("HIP_VISIBLE_DEVICES") or ""
    ids = [x for x in gpus.split(",") if x.strip()]
    if ids and len(ids) < n:
        raise RuntimeError(f"--nproc-per-pod {n} but the pod was given {len(ids)} GPU(s) ({gpus})")
    kids = {}

    def forward(signum, frame):
        for p in kids:
            try:
                os.killpg(p, signum)
            except ProcessLookupError:
                pass
    # forwarding is in place before the first fork, and the signals are held
    # while the loop forks: a SIGTERM during startup (pod deleted while its ranks
    # launch) reaches every rank already forked instead of killing the supervisor
    # with the default action and orphaning them
    sigs = {signal.SIGTERM, signal.SIGINT}
    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    signal.pthread_sigmask(signal.SIG_BLOCK, sigs)
    for i in range(n):
        env = jenv.torch_env(i, n)
        pid = os.fork()
        if pid == 0:
            os.setpgid(0, 0)
            signal.signal(signal.SIGTERM, signal.SIG_DFL)
            signal.signal(signal.SIGINT, signal.default_int_handler)
            signal.pthread_sigmask(signal.SIG_UNBLOCK, sigs)
            os.environ.update(env)
            os.environ["PDO_LOCAL_CHILD"] = "1"
            try:
                _hang_dump()
                rc = run_collective(args, jenv)
            except SystemExit as e:
                rc = e.code if isinstance(e.code, int) else 1
            except BaseException:
                import traceback
                traceback.print_exc()
                rc = 1
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(int(rc or 0))
        kids[pid] = i
        try:  # parent side too: no window where a forwarded signal misses the new group
            os.setpgid(pid, pid)
        except OSError:
            pass
    signal.pthread_sigmask(signal.SIG_UNBLOCK, sigs)
    log(f"pod {jenv.trainer_id}: {n} local ranks {env['WORLD_SIZE']}-world, pids {list(kids)}")
    rc = 0
    while kids:
        pid, status = os.wait()
        i = kids.pop(pid, None)
        if i is None:
            continue
        code = os.waitstatus_to_exitcode(status)
        code = 128 - code if code < 0 else code
        if code and not rc:
            rc = code
            log(f"local rank {i} exited {code}: stopping the other {len(kids)}")
            forward(signal.SIGTERM, None)
    return rc


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


def _hang_dump():
    hang_dump = float(os.environ.get("PDO_HANG_DUMP_S", "0") or 0)
    if hang_dump > 0:
        # hang diagnostics: every thread's Python stack to the pod log every N s
        # (a rank stuck in a collective shows where; no debugger attached)
        import faulthandler
        faulthandler.dump_traceback_later(hang_dump, repeat=True, file=sys.stderr)


def main(argv=None) -> int:
    args = parse_args(argv)
    from .env import JobEnv
    jenv = JobEnv.from_env()
    jenv.check_supported()
    log(f"role={jenv.role} id={jenv.trainer_id} mode={jenv.mode} elastic={jenv.elastic} workload={args.workload}")
    ps = jenv.mode == "PS" or args.workload in ("wide_deep", "deepfm") and jenv.pserver_endpoints
    if (args.nproc_per_pod > 1 and not ps and os.environ.get("PDO_LOCAL_CHILD") != "1"
            and not (jenv.elastic or args.elastic)):
        return spawn_local(args, jenv, argv)  # before any thread or HIP call in this process
    # elastic + --nproc-per-pod N: the agent below forks N fresh local ranks per generation
    _hang_dump()
    if ps:
        return run_ps(args, jenv)
    if (jenv.elastic or args.elastic) and not args.worker:
        from .elastic import run_agent
        return run_agent(args, jenv, argv if argv is not None else sys.argv[1:])
    return run_collective(args, jenv)


if __name__ == "__main__":
    sys.exit(main())
