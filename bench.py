#!/usr/bin/env python3
"""Headline benchmark: a *launched* GPT-2-medium PaddleJob on N MI355X.

BASELINE.json metric: "job-start->all-ranks-ready p50 (s); launched tokens/sec
at 1/2/4/8 MI355X".  Both halves are measured here, through the operator:

1. this process starts the native local backend in-process (object store +
   PaddleJob controller in ``fast`` mode + gang scheduler + kubelet-lite exec
   agent with its per-node warm launcher + pdo-kv) — the same C++ code as
   ``pdo-manager --backend=local`` (csrc/core);
2. **ready p50**: ``--ready-trials`` PaddleJobs of N ``noop`` ranks (one
   ``amd.com/gpu`` each) are created one after the other; a trial's latency is
   PaddleJob create → the last rank's readiness record in pdo-kv, where a rank
   is ready once its RCCL communicator is up (eager ``device_id`` init, even at
   one rank) and a warm-up all-reduce has completed (launch/bootstrap.py).
   Each trial starts on an idle node: the node's warm launcher has its
   per-GPU warm slot up (HIP initialised and RCCL's device code loaded in a
   process that then becomes the rank — launch/zygote.py); the job's own
   communicator (world size, rendezvous, rings) is built inside the measured
   interval.  ``--no-warm-slots`` measures without the slots;
3. **throughput**: one PaddleJob with ``worker.replicas=N`` whose ranks run
   ``pdo-launch --workload gpt2 --model gpt2-medium --batch 64 --seq 1024
   --bench``: W untimed steps, then exactly K timed steps bracketed by barrier +
   device synchronize; each rank publishes its elapsed time to pdo-kv and the
   MAX over ranks gives the whole-job tokens/s.

The reference's launch path being emulated is
controllers/paddlejob_controller.go:277-330 (pod creation → ConfigMap →
ordered release); its data plane is the launched job
(deploy/examples/resnet.yaml:14-25).  ``--compat-trials`` adds ready trials of
the reference-equivalent ``compat`` sequencing (cold interpreters, one mutation
per reconcile, busybox-style coordinator released by exec) for comparison.

Rank processes are spawned by the agent, never by torchrun: ``python bench.py
--gpus 8`` is a complete 8-GPU run.  Under the driver's
``torch.distributed.run --nproc-per-node N bench.py --gpus N`` the torchrun
rank 0 is the launcher and the other torchrun processes wait on a CPU (gloo)
barrier without touching the GPU.  This process never initialises HIP: GPUs are
counted from KFD sysfs, so the agent may fork+exec ranks from it.

Data: synthetic tokens generated on device each step; weights: random init.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import socket
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_METRIC = "job-start->all-ranks-ready p50 (s); launched tokens/sec at 1/2/4/8 MI355X"
# torchrun's contract variables: never inherited by the ranks this process launches
TORCHRUN_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                 "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT")


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks to launch (one MI355X each)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="gpt2", choices=["gpt2", "resnet50"],
                    help="gpt2 = the BASELINE headline (GPT-2-medium tokens/s); resnet50 = configs 2/3 (images/s)")
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--tiny", action="store_true", help=argparse.SUPPRESS)  # CPU tests: tiny resnet
    ap.add_argument("--micro-batch", type=int, default=int(os.environ.get("PDO_MICRO_BATCH", "0")),
                    help="per-rank batch (default 64 sequences for gpt2, 256 images for resnet50)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--ready-trials", type=int, default=10)
    ap.add_argument("--compat-trials", type=int, default=3,
                    help="ready trials in the reference-equivalent compat mode (the record's compat_ready)")
    ap.add_argument("--train-ready-trials", type=int, default=5,
                    help="ready trials of the headline workload itself (GPT-2 / ResNet ranks: model built on "
                         "the GPU and its initial weights broadcast, then ready) — the record's ready_train")
    ap.add_argument("--b2b-trials", type=int, default=5,
                    help="noop ready trials created back to back, without waiting for the node's warm slots "
                         "to re-warm (the record's ready_b2b)")
    ap.add_argument("--mode", default="fast", choices=["fast", "compat"])
    ap.add_argument("--no-zygote", action="store_true", help="cold interpreter per rank")
    ap.add_argument("--no-warm-slots", action="store_true",
                    help="zygote without GPU-warm slots (every rank inits HIP + RCCL from scratch)")
    ap.add_argument("--cpu", action="store_true", help="ranks on CPU (gloo) even if GPUs are present")
    ap.add_argument("--gpu-visibility", choices=["all", "isolate"], default="all",
                    help="node agent GPU exposure: all = every rank sees the node's GPUs and selects its own "
                         "(PDO_GPU_IDS, as torchrun-style launches; RCCL sees xGMI peers as local devices); "
                         "isolate = HIP_VISIBLE_DEVICES per pod, as a Kubernetes device plugin")
    ap.add_argument("--pod-layout", choices=["per-gpu", "one-pod"], default=os.environ.get("PDO_POD_LAYOUT", "per-gpu"),
                    help="per-gpu = N pods × 1 amd.com/gpu (the reference's layout, deploy/examples/resnet.yaml); "
                         "one-pod = 1 pod × N amd.com/gpu running --nproc-per-pod N local ranks (the Kubernetes "
                         "xGMI layout: under a device plugin only GPUs of one pod see each other)")
    ap.add_argument("--ops", choices=["hip", "torch"], default=os.environ.get("PDO_OPS", "hip"))
    ap.add_argument("--secondary-resnet", type=int, default=int(os.environ.get("PDO_BENCH_RESNET", "1")),
                    help="after the GPT-2 job (GPU or virtual-GPU nodes): a ResNet-50 job (configs 2/3: "
                         "deploy/examples/resnet.yaml, batch 256 per GPU, 20 timed steps) on the same N ranks, reported "
                         "under 'secondary' — 1: run it, 0: skip")
    ap.add_argument("--gang", choices=["auto", "on", "off"], default="auto",
                    help="Volcano gang scheduling of the benchmark jobs (config 4: PodGroup minMember=N, "
                         "reference controllers/paddlejob_helper.go:478-549): auto = on for N > 1")
    ap.add_argument("--timeout", type=float, default=900.0, help="per-job limit (s)")
    ap.add_argument("--keep", action="store_true", help="keep the sandbox (rank logs)")
    ap.add_argument("--ready-only", action="store_true", help="only the ready trials (prints their record)")
    # N ranks on ONE GPU over gloo (RCCL refuses two ranks per device): rehearses the
    # multi-rank launched GPU path (agent GPU accounting, DDP hooks over the HIP
    # kernels, per-rank records, comm diagnostics) on a 1-GPU box; not a benchmark
    ap.add_argument("--rehearse-shared-gpu", action="store_true", help=argparse.SUPPRESS)
    # with --cpu: the node offers N virtual GPUs (agent GPU accounting, one warm
    # slot per "GPU" in the zygote's CPU test mode, amd.com/gpu requests) while the
    # ranks run on CPU over gloo — the N-rank launched path's rehearsal (CPU tests)
    ap.add_argument("--virtual-gpus", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


class Launcher:
    """One in-process local backend; launches PaddleJobs and reads pdo-kv."""

    def __init__(self, mode, zygote, gpus, sandbox, extra_args=(), nproc=1, cpu_threads=0, volcano=False):
        from paddle_operator_amd.controller import LocalCluster
        from paddle_operator_amd.kv.client import KVClient

        self.port = _free_port()
        self.gpus = gpus
        self.sandbox = sandbox
        self.zygote = zygote
        self.extra_args = list(extra_args)
        self.nproc = nproc  # ranks per pod (--nproc-per-pod; amd.com/gpu per pod)
        self.cpu_threads = cpu_threads  # --virtual-gpus: CPU ranks behind GPU requests
        self.volcano = volcano
        self.cl = LocalCluster(mode=mode, agent="exec", sandbox_root=sandbox,
                               nodes=[{"name": "node0", "gpus": gpus}],
                               kv_endpoint=f"127.0.0.1:{self.port}", zygote=zygote, volcano=volcano)
        self.gang_log = {}  # job -> PodGroup observations (wait_records)
        self.cl.serve(f"127.0.0.1:{self.port}")
        self.cl.start()
        self.kv = KVClient(f"127.0.0.1:{self.port}")
        if zygote:
            t0 = time.time()
            # node warm-up (the zygote imports torch once), not part of any job's launch
            while not self.cl.zygotes_ready():
                if time.time() - t0 > 600:
                    raise RuntimeError("zygote not ready after 600 s; see " + os.path.join(sandbox, "zygote.log"))
                time.sleep(0.05)
            log(f"zygote ready in {time.time() - t0:.1f}s")

    def container(self, args, ops, scheduler=None):
        from paddle_operator_amd.api import types as T
        env = [{"name": "PYTHONPATH", "value": REPO}, {"name": "PDO_KV", "value": f"127.0.0.1:{self.port}"},
               {"name": "PDO_PYTHON", "value": sys.executable}, {"name": "PDO_OPS", "value": ops}]
        if not self.gpus or self.cpu_threads:
            env.append({"name": "OMP_NUM_THREADS", "value": str(self.cpu_threads or 2)})
        c = {"name": "paddle", "image": "pdo/launcher:rocm",
             "command": [os.path.join(REPO, "bin", "pdo-launch")] + list(args), "env": env}
        if self.gpus:
            c["resources"] = {"limits": {T.AMD_GPU: self.nproc}}
        return c

    def launch(self, name, ranks, args, ops, gang=False):
        """``gang``: the job goes through the Volcano path (PodGroup with
        minMember = pods, all-or-nothing binding by the gang scheduler); else,
        on a volcano-enabled cluster, it opts out with the default scheduler
        (builders.cpp without_volcano), as the ready trials do."""
        from paddle_operator_amd.api import types as T
        args = list(args) + self.extra_args
        if self.nproc > 1:
            args += ["--nproc-per-pod", str(self.nproc)]
        pods = ranks // self.nproc
        spec = {"containers": [self.container(args, ops)]}
        policy = None
        if self.volcano and gang:
            policy = {"minAvailable": pods, "queue": "default"}
            self.gang_log[name] = {"phases": [], "bound_before_inqueue": 0, "min_member": None}
        elif self.volcano:
            spec["schedulerName"] = "default-scheduler"
        job = T.paddlejob(name, worker={"replicas": pods, "template": {"spec": spec}},
                          clean_pod_policy="Always", scheduling_policy=policy)
        t0 = time.time()
        self.cl.create(job)
        return t0

    def wait_records(self, name, kind, n, timeout):
        prefix = f"/pdo/default-{name}/{kind}/"
        deadline = time.time() + timeout
        recs = {}
        beat = time.time() + 30
        while time.time() < deadline:
            recs = self.kv.get_prefix(prefix)
            if name in self.gang_log:
                self._watch_gang(name)
            if len(recs) >= n:
                return [json.loads(v) for v in recs.values()]
            phase = ((self.cl.job(name) or {}).get("status") or {}).get("phase")
            if phase == "Failed":
                break
            if time.time() > beat:  # progress line for long jobs (many ranks, slow steps)
                log(f"{name}: {len(recs)}/{n} {kind} records, phase {phase}")
                beat = time.time() + 30
            time.sleep(0.005)
        self.dump_logs(name)
        raise RuntimeError(f"{name}: {len(recs)}/{n} {kind} records (phase "
                           f"{((self.cl.job(name) or {}).get('status') or {}).get('phase')})")

    def _watch_gang(self, name):
        """PodGroup phase sequence, and whether any pod was bound to a node
        while its PodGroup was not yet admitted (Inqueue / Running)."""
        g = self.gang_log[name]
        if g.get("admitted"):
            return
        pg = self.cl.get("PodGroup", name)
        if pg is None:
            return
        ph = (pg.get("status") or {}).get("phase") or "Pending"
        g["min_member"] = (pg.get("spec") or {}).get("minMember")
        if not g["phases"] or g["phases"][-1] != ph:
            g["phases"].append(ph)
        bound = sum(bool((p.get("spec") or {}).get("nodeName")) for p in self.cl.pods(name))
        g["bound_pods"] = bound
        if bound and ph not in ("Inqueue", "Running"):
            g["bound_before_inqueue"] += 1
        g["admitted"] = ph == "Running" and bound == g["min_member"]

    def dump_logs(self, name, tail=int(os.environ.get("PDO_BENCH_LOG_TAIL", "4000"))):
        import glob
        for path in sorted(glob.glob(os.path.join(self.sandbox, "*", f"default_{name}-*", "*.log")) +
                           glob.glob(os.path.join(self.sandbox, "*", "zygote.log"))):
            try:
                with open(path) as f:
                    log(f"--- {os.path.relpath(path, self.sandbox)} (tail) ---\n{f.read()[-tail:]}")
            except OSError:
                pass

    def finish(self, name, timeout=120):
        from paddle_operator_amd.api import types as T
        ok = self.cl.wait_phase(name, "Completed", timeout=timeout)
        if not ok:
            self.dump_logs(name)
            raise RuntimeError(f"{name}: not Completed "
                               f"({((self.cl.job(name) or {}).get('status') or {}).get('phase')})")
        self.cl.delete(T.KIND, name)
        self.cl.wait(lambda: self.cl.job(name) is None and not self.cl.pods(name), timeout=60)

    def ready_trial(self, name, ranks, timeout, args=None, ops="torch", wait_warm=True):
        """Create → the last rank's readiness record.  ``args``: the rank's
        workload (default a noop rank); ``wait_warm``: start on an idle node
        whose warm slots are all up (False: right after the previous job)."""
        if wait_warm and self.zygote and self.gpus and not self.cl.wait_warm(timeout=120):
            log("warm slots not all up after 120 s; trial runs with what is there")
        t0 = self.launch(name, ranks, (args or ["--workload", "noop"]) + ["--exit-after-ready"], ops)
        rs = self.wait_records(name, "ready", ranks, timeout)
        self.finish(name)
        slow = max(rs, key=lambda r: r["t_ready"])
        return {"ready_s": slow["t_ready"] - t0,
                "pg_s": max(r["t_pg"] - r["t_start"] for r in rs),
                "proc_start_s": min(r["t_start"] for r in rs) - t0,
                "warm": sum(bool(r.get("warm_slot")) for r in rs) / len(rs),
                "phases": slow.get("phases") or {}}

    def stop(self):
        self.cl.stop()


def ready_stats(trials):
    v = [t["ready_s"] for t in trials]
    med = lambda xs: round(statistics.median(xs), 4)  # noqa: E731
    out = {"p50": med(v), "min": round(min(v), 4), "max": round(max(v), 4), "trials": len(v),
           "pg_init_p50": med([t["pg_s"] for t in trials]),
           "proc_start_p50": med([t["proc_start_s"] for t in trials]),
           "warm_slot_fraction": round(sum(t["warm"] for t in trials) / len(trials), 3)}
    # where the slowest rank's time went (medians over trials): create → process start
    # is the control plane + warm launcher; the rest is inside the rank
    keys = set().union(*(t["phases"].keys() for t in trials))
    out["rank_phases_p50"] = {k: med([t["phases"].get(k, 0.0) for t in trials]) for k in sorted(keys)}
    return out


def _comm_summary(rs):
    """Worst rank's exposed all-reduce time per step and slowest bucket all-reduce."""
    cs = [r["comm"] for r in rs if r.get("comm")]
    if not cs:
        return None
    out = {"ranks": len(cs), "allreduce_bytes": cs[0].get("allreduce_bytes"),
           "allreduce_busbw_GBps_min": min(c["allreduce_busbw_GBps"] for c in cs)}
    # size sweep: the slowest rank per size (every rank times the same collectives)
    sw = [c["allreduce_sweep"] for c in cs if c.get("allreduce_sweep")]
    if sw:
        out["allreduce_sweep"] = [{"bytes": p["bytes"], "busbw_GBps": min(s[i]["busbw_GBps"] for s in sw),
                                   "us": max(s[i]["us"] for s in sw)} for i, p in enumerate(sw[0])]
        best = max(p["busbw_GBps"] for p in out["allreduce_sweep"])
        out["knee_bytes"] = next(p["bytes"] for p in out["allreduce_sweep"] if p["busbw_GBps"] >= 0.9 * best)
    if cs[0].get("buckets"):
        out["buckets"] = cs[0]["buckets"]
    ipc = [c["ipc_gbps"] for c in cs if "ipc_gbps" in c]
    if ipc:
        out["ipc_gbps"] = ipc
    ex = [c["exposed_ms"] for c in cs if "exposed_ms" in c]
    if ex:
        out["exposed_ms_max"] = max(ex)
        out["nosync_step_ms_max"] = max(c["nosync_step_ms"] for c in cs if "nosync_step_ms" in c)
    return out


def _gang_summary(g):
    if not g:
        return None
    return {"podgroup_min_member": g.get("min_member"), "podgroup_phases": g.get("phases"),
            "bound_pods": g.get("bound_pods"), "bound_before_inqueue": g.get("bound_before_inqueue"),
            "scheduler": "volcano (pdo gang scheduler)"}


def orchestrate(a):
    from paddle_operator_amd.models.gpt2 import GPT2Config
    from paddle_operator_amd.utils.topology import gpu_count

    N = a.gpus
    if not a.micro_batch:
        a.micro_batch = 64 if a.workload == "gpt2" else 256
    detected = 0 if a.cpu else gpu_count()
    extra_args = []
    if a.rehearse_shared_gpu:
        if not detected:
            log("--rehearse-shared-gpu needs a GPU")
            return 2
        # every agent GPU index maps to physical GPU 0; no warm slots (one per physical GPU)
        os.environ["HIP_VISIBLE_DEVICES"] = ",".join(["0"] * N)
        os.environ["PDO_WARM_SLOTS"] = "0"
        a.no_warm_slots = True
        os.environ.setdefault("PDO_HANG_DUMP_S", "60")  # rank stacks in the pod logs (launch/run.py)
        extra_args = ["--backend", "gloo"]
        detected = N
    if a.virtual_gpus:
        if not a.cpu:
            log("--virtual-gpus needs --cpu")
            return 2
        os.environ["PDO_SLOT_TEST"] = "cpu"  # warm slots without HIP (launch/zygote.py)
        extra_args = ["--backend", "gloo"]
        detected = N
    if detected and detected < N:
        log(f"--gpus {N} but only {detected} GPU(s) visible")
        return 2
    gpus = N if detected else 0  # the job asks for N amd.com/gpu; the node offers exactly those
    if gpus:
        # read by the in-process agent (csrc/core/agent.cpp) and its warm launcher
        os.environ["PDO_GPU_VISIBILITY"] = "isolate" if a.rehearse_shared_gpu else a.gpu_visibility
        # warm slots per GPU: three (back-to-back jobs start warm: launch/zygote.py
        # slots_per_gpu) up to 2 GPUs; one above, so ranks + slots stay at ≤ 2
        # processes per GPU on a full node
        os.environ.setdefault("PDO_SLOTS_PER_GPU", "3" if N <= 2 else "1")
    sandbox = tempfile.mkdtemp(prefix="pdo-bench-")
    if a.no_warm_slots:
        os.environ["PDO_WARM_SLOTS"] = "0"  # read by the agent when it starts the zygote
    out = {}
    try:
        nproc = N if a.pod_layout == "one-pod" else 1
        gang = a.gang == "on" or (a.gang == "auto" and N > 1)
        L = Launcher(a.mode, not a.no_zygote, gpus, os.path.join(sandbox, a.mode), extra_args, nproc,
                     cpu_threads=1 if a.virtual_gpus else 0, volcano=gang)
        try:
            trials = []
            for t in range(a.ready_trials):
                trials.append(L.ready_trial(f"ready-{t}", N, a.timeout))
            out["ready"] = ready_stats(trials) if trials else None
            if trials:
                log(f"ready p50 {out['ready']['p50']}s over {len(trials)} trials ({N} ranks)")
            if L.zygote and gpus:
                # the warm slots' resident footprint (HIP context + RCCL code), per GPU
                st = L.cl.zygote_status()
                out["warm_slots"] = {node: {d: {k: sl.get(k) for k in ("mem_mb", "mem_mb_before_rccl", "warm_s", "n", "n_ready")}
                                            for d, sl in (z or {}).get("slots", {}).items()}
                                     for node, z in st.items()}
            if a.b2b_trials and not a.ready_only:
                bt = [L.ready_trial(f"b2b-{t}", N, a.timeout, wait_warm=False) for t in range(a.b2b_trials)]
                out["ready_b2b"] = ready_stats(bt)
                log(f"back-to-back ready p50 {out['ready_b2b']['p50']}s "
                    f"(warm-slot fraction {out['ready_b2b']['warm_slot_fraction']})")
            if a.ready_only:
                print(json.dumps({"metric": "job-start->all-ranks-ready p50", "unit": "s", "n_gpus": N,
                                  "mode": a.mode, "zygote": not a.no_zygote, "ready": out.get("ready"),
                                  "env": {k: v for k, v in os.environ.items()
                                          if k.startswith(("NCCL_", "RCCL_", "HSA_", "HIP_", "PDO_"))}}),
                      flush=True)
                return 0
            if os.environ.get("PDO_BENCH_PS"):
                import psutil
                kids = psutil.Process().children(recursive=True)
                log(f"{len(kids)} descendant processes before the bench job: " +
                    "; ".join(f"{k.pid} {' '.join(k.cmdline()[:3])[-60:]}" for k in kids))
            name = f"{a.workload}-bench"
            if a.workload == "gpt2":
                wl = ["--workload", "gpt2", "--model", a.model, "--batch", str(a.micro_batch), "--seq", str(a.seq)]
            else:
                wl = ["--workload", "resnet50", "--batch", str(a.micro_batch)] + (["--tiny"] if a.tiny else [])
            if a.train_ready_trials:
                # ready-to-train: the headline workload's ranks, model built and weights broadcast
                tt = [L.ready_trial(f"train-ready-{t}", N, a.timeout, args=list(wl), ops=a.ops)
                      for t in range(a.train_ready_trials)]
                out["ready_train"] = ready_stats(tt)
                log(f"ready-to-train p50 {out['ready_train']['p50']}s over {len(tt)} {a.workload} jobs")
            wl += ["--steps", str(a.steps), "--warmup", str(a.warmup), "--bench", "--timeout", "600"]
            t0 = L.launch(name, N, wl, a.ops, gang=gang)
            rs = L.wait_records(name, "bench", N, a.timeout)
            L.finish(name)
            out["bench"] = rs
            out["bench_ready_s"] = max(r["t_ready"] for r in rs) - t0
            if gang:
                out["gang"] = L.gang_log.get(name)
            if a.workload == "gpt2" and a.secondary_resnet and gpus:
                # the reference's own example workload (deploy/examples/resnet.yaml, config 3 at
                # N = 8) on the same N ranks in the same driver run; a failure here never costs
                # the headline record
                try:
                    if a.virtual_gpus:  # CPU rehearsal: the tiny ResNet, as --workload resnet50 --tiny
                        wl2 = ["--workload", "resnet50", "--tiny", "--batch", "2", "--steps", "2", "--warmup", "1"]
                    else:
                        wl2 = ["--workload", "resnet50", "--batch", "256", "--steps", "20", "--warmup", "5"]
                    wl2 += ["--bench", "--timeout", "600"]
                    L.launch("resnet50-bench", N, wl2, a.ops, gang=gang)
                    out["resnet"] = L.wait_records("resnet50-bench", "bench", N, min(a.timeout, 300.0))
                    out["resnet_wl"] = wl2
                    L.finish("resnet50-bench")
                    if gang:
                        out["resnet_gang"] = L.gang_log.get("resnet50-bench")
                except Exception as e:  # noqa: BLE001
                    out["resnet_error"] = f"{type(e).__name__}: {e}"
                    log(f"secondary ResNet-50 job failed: {out['resnet_error']}")
        finally:
            L.stop()
        if a.compat_trials:
            C = Launcher("compat", False, gpus, os.path.join(sandbox, "compat"), extra_args, nproc)
            try:
                ct = [C.ready_trial(f"compat-{t}", N, a.timeout) for t in range(a.compat_trials)]
            finally:
                C.stop()
            out["compat_ready"] = ready_stats(ct)
    finally:
        if a.keep:
            log(f"sandbox kept: {sandbox}")
        else:
            shutil.rmtree(sandbox, ignore_errors=True)

    rs = out["bench"]
    dt = max(r["seconds"] for r in rs)  # max over ranks
    items = sum(r["tokens_per_step_rank"] for r in rs) * a.steps
    rate = items / dt
    common = {
        "n_gpus": N, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None,  # BASELINE.json publishes no number ("published": {})
        "dtype": "bf16",
    }
    pods = N if a.pod_layout == "per-gpu" else 1
    launch = (f"PaddleJob worker.replicas={pods} x {N // pods} GPU, planner={a.mode}, zygote={not a.no_zygote}, "
              f"warm_slots={not a.no_zygote and not a.no_warm_slots and bool(gpus)}, "
              f"gpu_visibility={os.environ.get('PDO_GPU_VISIBILITY', 'isolate') if gpus else 'cpu'}"
              + (f", gang=volcano PodGroup minMember={pods}" if out.get("gang") else ""))
    extra = {
        "baseline_metric": BASELINE_METRIC,
        "ready_p50_s": out["ready"]["p50"] if out.get("ready") else None,
        "ready": out.get("ready"),
        # the headline workload's own create → every rank past its initial weight broadcast
        "ready_train": out.get("ready_train"),
        # noop jobs created back to back (warm slots may still be re-warming)
        "ready_b2b": out.get("ready_b2b"),
        "warm_slots": out.get("warm_slots"),
        "compat_ready": out.get("compat_ready"),
        "job_ready_s": round(out["bench_ready_s"], 3),
        "final_loss": rs[0].get("loss"),
        "max_mem_gb": max((r.get("max_mem_gb") or 0) for r in rs),
        # N > 1: measured after the timed region by every rank (launch/run.py _comm_diag)
        "comm": _comm_summary(rs),
        # Volcano gang path (N > 1): the PodGroup's minMember and the phases it went
        # through; bound_before_inqueue counts polls that saw a pod bound before admission
        "gang": _gang_summary(out.get("gang")),
    }
    dev = "cpu/gloo" if not gpus else rs[0].get("gpu_name", "gpu")
    if a.workload == "gpt2":
        cfg = GPT2Config.named(a.model)
        flops_gpu = cfg.flops_per_token(a.seq) * rate / N
        rec = {"metric": "launched tokens/sec (GPT-2-medium PaddleJob through the pdo operator, collective DP over RCCL)",
               "value": round(rate, 1), "unit": "tokens/s", **common,
               "data": "synthetic (on-device random tokens), random-init weights",
               "config": {"model": a.model, "global_batch": a.micro_batch * N, "micro_batch_per_gpu": a.micro_batch,
                          "seq_len": a.seq, "parallelism": f"dp{N}" + ("-shared-gpu-gloo" if a.rehearse_shared_gpu else ""),
                          "launch": launch, "pod_layout": f"{pods}x{N // pods}",
                          "grad_reduce": rs[0].get("grad_reduce"), "buckets": rs[0].get("buckets"), "ops": a.ops,
                          "device": dev},
               **extra,
               "gpt2_job_ready_s": extra["job_ready_s"],
               "model_tflops_per_gpu": round(flops_gpu / 1e12, 1),
               "mfu_vs_2.5PF_dense": round(flops_gpu / 2.5e15, 4)}
        if out.get("resnet"):
            r2, wl2 = out["resnet"], out["resnet_wl"]
            st2, mb2 = int(wl2[wl2.index("--steps") + 1]), int(wl2[wl2.index("--batch") + 1])
            dt2 = max(r["seconds"] for r in r2)
            rate2 = sum(r["tokens_per_step_rank"] for r in r2) * st2 / dt2
            rec["secondary"] = {
                "metric": "launched images/sec (ResNet-50 PaddleJob through the pdo operator, collective DP over RCCL)",
                "value": round(rate2, 1), "unit": "images/s", "n_gpus": N, "steps": st2,
                "warmup": int(wl2[wl2.index("--warmup") + 1]),
                "ms_per_step": round(dt2 / st2 * 1e3, 3), "dtype": "bf16" if not a.virtual_gpus else "fp32",
                "data": "synthetic (on-device random 224x224 images and labels), random-init weights",
                "config": {"model": "resnet18-like-tiny (CPU rehearsal)" if a.virtual_gpus else "resnet50", "global_batch": mb2 * N,
                           "micro_batch_per_gpu": mb2, "resolution": 32 if a.virtual_gpus else 224,
                           "parallelism": f"dp{N}", "pod_layout": f"{pods}x{N // pods}",
                           "step": "hip-graph replay" if all(r.get("hip_graph") for r in r2) else "eager"},
                "max_mem_gb": max((r.get("max_mem_gb") or 0) for r in r2),
                "comm": _comm_summary(r2), "gang": _gang_summary(out.get("resnet_gang"))}
        elif out.get("resnet_error"):
            rec["secondary"] = {"error": out["resnet_error"]}
    else:
        rec = {"metric": "launched images/sec (ResNet-50 PaddleJob through the pdo operator, collective DP over RCCL)",
               "value": round(rate, 1), "unit": "images/s", **common,
               "data": "synthetic (on-device random 224x224 images and labels), random-init weights",
               "config": {"model": "resnet50", "global_batch": a.micro_batch * N, "micro_batch_per_gpu": a.micro_batch,
                          "resolution": 224, "parallelism": f"dp{N}", "launch": launch,
                          "pod_layout": f"{pods}x{N // pods}",
                          "grad_reduce": rs[0].get("grad_reduce"), "buckets": rs[0].get("buckets"), "device": dev},
               **extra}
    print(json.dumps(rec), flush=True)
    return 0


def main(argv=None):
    a = parse_args(argv)
    tr_world = int(os.environ.get("WORLD_SIZE", "1"))
    tr_rank = int(os.environ.get("RANK", "0"))
    if tr_world > 1:
        # the driver's torchrun wrapper: rank 0 launches the job, the others
        # only keep torchrun's world alive (CPU gloo barrier, no GPU)
        import datetime

        import torch.distributed as dist
        dist.init_process_group("gloo", rank=tr_rank, world_size=tr_world,
                                timeout=datetime.timedelta(seconds=7200))
        rc = 0
        if tr_rank == 0:
            for k in TORCHRUN_VARS:
                os.environ.pop(k, None)
            for k in [k for k in os.environ if k.startswith("TORCHELASTIC_")]:
                os.environ.pop(k, None)
            try:
                rc = orchestrate(a)
            except Exception as e:
                log(f"failed: {e}")
                rc = 1
        import torch
        t = torch.tensor([rc], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.destroy_process_group()
        return int(t.item())
    try:
        return orchestrate(a)
    except Exception as e:
        log(f"failed: {e}")
        return 1


if __name__ == "__main__":
    sys.exit(main())
