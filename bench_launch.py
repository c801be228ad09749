"""Job-launch latency benchmark: PaddleJob create → all ranks ready (p50).

BASELINE.json's first headline metric.  Drives the native local backend
(object store + controller + gang scheduler + kubelet-lite exec agent +
pdo-kv) with real ``pdo-launch`` rank processes, in both planner modes:

* ``compat`` — the reference's sequencing (one mutation per reconcile, 1 s
  requeues, ConfigMap barrier, busybox-style coordinator init container
  released by exec ``touch goon`` in ps→worker→heter order, phase lag);
* ``fast``   — pdo's path (batched creates, event-driven requeues, no init
  barrier: ranks rendezvous on the RCCL TCPStore directly);
* ``fast+zygote`` — plus the per-node warm launcher: ``bin/pdo-launch``
  forks the rank from a pre-imported interpreter (launch/zygote.py) instead
  of paying Python + ``import torch`` start-up per rank.

Every mode uses the same container entry point (``bin/pdo-launch``); without
a zygote it execs ``python -m paddle_operator_amd.launch``.

A rank is *ready* once its process group is up, the warm-up all-reduce has
completed and it wrote ``/pdo/<job>/ready/<rank>`` to pdo-kv
(launch/bootstrap.py); latency = max over ranks of that wall-clock stamp −
the wall-clock time just before the PaddleJob was created.

    python bench_launch.py --ranks 1,2,4,8 --trials 10            # GPUs if present, else gloo/CPU
    python bench_launch.py --modes fast --ranks 1 --workload resnet50

Prints one JSON line per (mode, ranks) and a summary line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gpu_count():
    # KFD sysfs, never HIP: this process's agent fork+execs every rank
    from paddle_operator_amd.utils.topology import gpu_count
    return gpu_count()


def run(mode, ranks, trials, workload, gpus, sandbox, timeout=180.0, extra_args=()):
    from paddle_operator_amd.api import types as T
    from paddle_operator_amd.controller import LocalCluster
    from paddle_operator_amd.kv.client import KVClient

    port = _free_port()
    node = {"name": "node0", "gpus": gpus}
    planner, _, zyg = mode.partition("+")
    cl = LocalCluster(mode=planner, agent="exec", sandbox_root=os.path.join(sandbox, mode), nodes=[node],
                      kv_endpoint=f"127.0.0.1:{port}", zygote=zyg == "zygote")
    cl.serve(f"127.0.0.1:{port}")
    cl.start()
    t_z = time.time()
    while not cl.zygotes_ready() and time.time() - t_z < 120:  # node warm-up, not part of a job's launch
        time.sleep(0.05)
    kv = KVClient(f"127.0.0.1:{port}")
    env = [{"name": "PYTHONPATH", "value": REPO}, {"name": "PDO_KV", "value": f"127.0.0.1:{port}"},
           {"name": "OMP_NUM_THREADS", "value": "4"}, {"name": "PDO_PYTHON", "value": sys.executable}]
    args = ["--workload", workload, "--exit-after-ready"] + list(extra_args)
    if workload != "noop":
        args += ["--steps", "1"]
    cont = {"name": "paddle", "image": "pdo/launcher:rocm",
            "command": [os.path.join(REPO, "bin", "pdo-launch")] + args, "env": env}
    if gpus:
        cont["resources"] = {"limits": {T.AMD_GPU: 1}}
    out = []
    try:
        for t in range(trials):
            name = f"lj-{mode}-{ranks}-{t}"
            job = T.paddlejob(name, worker={"replicas": ranks, "template": {"spec": {"containers": [cont]}}},
                              clean_pod_policy="Always")
            prefix = f"/pdo/default-{name}/ready/"
            t0 = time.time()
            cl.create(job)
            recs = {}
            deadline = t0 + timeout
            while time.time() < deadline:
                recs = kv.get_prefix(prefix)
                if len(recs) >= ranks:
                    break
                time.sleep(0.005)
            t_seen = time.time()
            if len(recs) < ranks:
                raise RuntimeError(f"{name}: only {len(recs)}/{ranks} ranks ready after {timeout}s")
            rs = [json.loads(v) for v in recs.values()]
            t_ready = max(r["t_ready"] for r in rs)
            out.append({"ready_s": t_ready - t0, "seen_s": t_seen - t0,
                        "proc_start_s": min(r["t_start"] for r in rs) - t0,
                        "pg_s": max(r["t_pg"] - r["t_start"] for r in rs)})
            cl.wait_phase(name, "Completed", timeout=60)
            cl.delete(T.KIND, name)
            cl.wait(lambda: cl.job(name) is None and not cl.pods(name), timeout=60)
    finally:
        cl.stop()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1")
    ap.add_argument("--trials", type=int, default=10)
    ap.add_argument("--modes", default="compat,fast,fast+zygote",
                    help="planner mode, optionally +zygote (per-node warm launcher)")
    ap.add_argument("--workload", default="noop", choices=["noop", "resnet50", "gpt2"])
    ap.add_argument("--gpus", type=int, default=-1, help="GPUs on the node (-1: detect)")
    ap.add_argument("--timeout", type=float, default=180.0)
    a = ap.parse_args(argv)
    gpus = _gpu_count() if a.gpus < 0 else a.gpus
    results = []
    with tempfile.TemporaryDirectory(prefix="pdo-launch-bench-") as sb:
        for mode in a.modes.split(","):
            for n in [int(x) for x in a.ranks.split(",")]:
                if gpus and n > gpus:
                    print(f"# skip ranks={n}: only {gpus} GPUs", file=sys.stderr)
                    continue
                tr = run(mode, n, a.trials, a.workload, gpus, sb, a.timeout)
                ready = [x["ready_s"] for x in tr]
                rec = {"metric": "job-start->all-ranks-ready p50", "mode": mode, "ranks": n,
                       "value": round(statistics.median(ready), 3), "unit": "s", "higher_is_better": False,
                       "min": round(min(ready), 3), "max": round(max(ready), 3), "trials": len(ready),
                       "proc_start_p50": round(statistics.median(x["proc_start_s"] for x in tr), 3),
                       "pg_init_p50": round(statistics.median(x["pg_s"] for x in tr), 3),
                       "backend": "nccl" if gpus else "gloo", "workload": a.workload}
                print(json.dumps(rec), flush=True)
                results.append(rec)
    by = {}
    for r in results:
        by.setdefault(r["ranks"], {})[r["mode"]] = r["value"]
    print(json.dumps({"summary": "ready p50 (s) by ranks", "by_ranks": by}), flush=True)


if __name__ == "__main__":
    main()
