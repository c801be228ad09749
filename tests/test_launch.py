"""pdo-launch on CPU: env contract, collective (gloo world 2), PS mode,
checkpoint/resume and the elastic agent (2 → 3 ranks re-rendezvous).

The reference has no launcher (the Paddle image brings one); these tests pin
the contract the operator's ConfigMap/env emits (SURVEY Appendix A,
controllers/paddlejob_helper.go:215-377) to what pdo-launch consumes.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from paddle_operator_amd.launch.env import STORE_PORT_OFFSET, JobEnv

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port_block(n=40):
    """A base port p with p..p+n free (best effort).

    Drawn below the kernel's ephemeral range (32768+) so that client sockets
    of concurrently running tests (pytest-xdist) cannot land inside the block
    between this probe and the launcher's bind."""
    import random
    rng = random.Random(os.getpid() ^ time.time_ns())
    for _ in range(200):
        p = rng.randrange(12000, 32000 - n)
        ok = True
        for q in range(p, p + n):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", q))
            except OSError:
                ok = False
            finally:
                t.close()
            if not ok:
                break
        if ok:
            return p
    raise RuntimeError("no free port block")


def launch(env_extra, args, log_path):
    env = dict(os.environ)
    env.update({"OMP_NUM_THREADS": "2", "PYTHONPATH": REPO, "PDO_OPS": "torch"})
    env.update({k: str(v) for k, v in env_extra.items()})
    f = open(log_path, "w")
    p = subprocess.Popen([sys.executable, "-m", "paddle_operator_amd.launch"] + args, env=env, cwd=REPO,
                         stdout=f, stderr=subprocess.STDOUT, start_new_session=True)
    p._log = log_path
    return p


def wait_all(procs, timeout=240):
    t_end = time.time() + timeout
    for p in procs:
        try:
            p.wait(max(1, t_end - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    os.killpg(q.pid, 9)
            raise AssertionError("launcher timed out:\n" + "\n".join(open(q._log).read()[-3000:] for q in procs))
    return [p.returncode for p in procs]


def records(path, tag):
    out = []
    for line in open(path):
        if line.startswith(tag + " "):
            out.append(json.loads(line[len(tag) + 1:]))
    return out


# ----------------------------------------------------------------------------- env contract
def test_env_collective_mapping():
    e = JobEnv.from_env({"PADDLE_TRAINER_ID": "1", "TRAINING_ROLE": "TRAINER", "POD_IP": "10.0.0.2",
                         "PADDLE_PORT": "2379", "PADDLE_TRAINERS_NUM": "2",
                         "PADDLE_TRAINER_ENDPOINTS": "10.0.0.1:2379,10.0.0.2:2379"})
    assert e.mode == "Collective"
    t = e.torch_env(local_rank=1, nproc_per_pod=2)
    assert t == {"RANK": "3", "WORLD_SIZE": "4", "LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "2",
                 "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": str(2379 + STORE_PORT_OFFSET)}


def test_env_ps_mapping():
    base = {"PADDLE_PSERVERS_IP_PORT_LIST": "10.0.0.1:2379,10.0.0.2:2379",
            "PADDLE_TRAINER_ENDPOINTS": "10.0.0.3:2379,10.0.0.4:2379,10.0.0.5:2379", "PADDLE_TRAINERS_NUM": "3"}
    ps1 = JobEnv.from_env(dict(base, TRAINING_ROLE="PSERVER", PADDLE_TRAINER_ID="1"))
    tr2 = JobEnv.from_env(dict(base, PADDLE_TRAINING_ROLE="TRAINER", PADDLE_TRAINER_ID="2"))
    assert ps1.mode == tr2.mode == "PS"
    assert ps1.ps_world() == (1, 5, "10.0.0.1:2379")
    assert tr2.ps_world() == (4, 5, "10.0.0.1:2379")


def test_env_single_and_elastic():
    assert JobEnv.from_env({}).mode == "Single"
    e = JobEnv.from_env({"PADDLE_ELASTIC_JOB_ID": "ns-job", "PADDLE_ELASTIC_NP": "4",
                         "PADDLE_ELASTIC_SERVER": "127.0.0.1:2379", "PADDLE_ELASTIC_TIMEOUT": "60"})
    assert e.elastic and e.mode == "Collective" and e.elastic_np == 4
    assert e.kv_endpoints() == "127.0.0.1:2379" and e.job_key() == "ns-job"


# ----------------------------------------------------------------------------- collective
def _collective_env(rank, world, base):
    eps = ",".join(f"127.0.0.1:{base + 20 * i}" for i in range(world))
    return {"PADDLE_TRAINER_ID": rank, "PADDLE_TRAINER_ENDPOINTS": eps, "PADDLE_TRAINERS_NUM": world,
            "POD_IP": "127.0.0.1", "PADDLE_PORT": base + 20 * rank, "TRAINING_ROLE": "TRAINER"}


@pytest.mark.parametrize("workload", ["resnet50", "gpt2"])
def test_collective_gloo_world2(tmp_path, workload):
    base = free_port_block()
    procs = [launch(_collective_env(r, 2, base), ["--workload", workload, "--tiny", "--steps", "4", "--log-every", "2",
                                                  "--seq", "128"], tmp_path / f"r{r}.log") for r in range(2)]
    assert wait_all(procs) == [0, 0], open(tmp_path / "r0.log").read()[-3000:]
    for r in range(2):
        ready = records(tmp_path / f"r{r}.log", "PDO_READY")
        done = records(tmp_path / f"r{r}.log", "PDO_DONE")
        assert ready and ready[0]["rank"] == r and ready[0]["world"] == 2 and ready[0]["backend"] == "gloo"
        assert done and done[0]["steps"] == 4


def test_collective_checkpoint_resume(tmp_path):
    base = free_port_block()
    ck = tmp_path / "ckpt"
    args = ["--workload", "gpt2", "--tiny", "--seq", "64", "--ckpt-dir", str(ck), "--ckpt-every", "2"]
    procs = [launch(_collective_env(r, 2, base), args + ["--steps", "4"], tmp_path / f"a{r}.log") for r in range(2)]
    assert wait_all(procs) == [0, 0], open(tmp_path / "a0.log").read()[-3000:]
    assert sorted(os.listdir(ck)) == ["ckpt-00000002.pt", "ckpt-00000004.pt"]
    # restart at world size 1: resumes from step 4, runs to 6
    p = launch(_collective_env(0, 1, base), args + ["--steps", "6"], tmp_path / "b.log")
    assert wait_all([p]) == [0], open(tmp_path / "b.log").read()[-3000:]
    ready = records(tmp_path / "b.log", "PDO_READY")[0]
    done = records(tmp_path / "b.log", "PDO_DONE")[0]
    assert ready["resume_step"] == 4 and done["steps"] == 2 and done["final_step"] == 6


# ----------------------------------------------------------------------------- parameter server
@pytest.mark.parametrize("workload", ["wide_deep", "deepfm"])
def test_ps_mode_wide_deep(tmp_path, workload):
    base = free_port_block()
    common = {"PADDLE_PSERVERS_IP_PORT_LIST": f"127.0.0.1:{base}",
              "PADDLE_TRAINER_ENDPOINTS": f"127.0.0.1:{base + 20},127.0.0.1:{base + 40}",
              "PADDLE_TRAINERS_NUM": 2, "PADDLE_WITH_GLOO": 1,
              "PADDLE_GLOO_HTTP_ENDPOINT": f"127.0.0.1:{base + 18}"}
    args = ["--workload", workload, "--tiny", "--steps", "60", "--batch", "256"]
    procs = [launch(dict(common, TRAINING_ROLE="PSERVER", PADDLE_TRAINER_ID=0), args, tmp_path / "ps0.log")]
    procs += [launch(dict(common, TRAINING_ROLE="TRAINER", PADDLE_TRAINER_ID=i), args, tmp_path / f"t{i}.log")
              for i in range(2)]
    assert wait_all(procs) == [0, 0, 0], open(tmp_path / "t0.log").read()[-3000:]
    for i in range(2):
        d = records(tmp_path / f"t{i}.log", "PDO_DONE")[0]
        assert d["last_loss"] < d["first_loss"] - 0.05, d  # the shared model learns
        assert d["server_stats"][0]["pushes"] >= 60
    assert records(tmp_path / "ps0.log", "PDO_READY")[0]["backend"] == "rpc+gloo"


# ----------------------------------------------------------------------------- elastic
def test_elastic_scale_out_reforms_world(tmp_path):
    core = pytest.importorskip("paddle_operator_amd._pdo_core")
    from paddle_operator_amd.kv.client import KVClient

    srv = core.KVServer("127.0.0.1:0")
    ep = f"127.0.0.1:{srv.port}"
    kv = KVClient(ep)
    base = free_port_block(80)
    ck = tmp_path / "ckpt"
    args = ["--workload", "resnet50", "--tiny", "--steps", "60", "--ckpt-dir", str(ck), "--ckpt-every", "5",
            "--throttle-ms", "60", "--log-every", "20"]

    def agent(i, np_):
        return launch({"PADDLE_ELASTIC_JOB_ID": "default-ej", "PADDLE_ELASTIC_NP": np_,
                       "PADDLE_ELASTIC_SERVER": ep, "PADDLE_ELASTIC_TIMEOUT": 60, "PADDLE_TRAINER_ID": i,
                       "POD_IP": "127.0.0.1", "PADDLE_PORT": base + 20 * i, "PDO_ELASTIC_TTL": 3},
                      args, tmp_path / f"e{i}.log")

    procs = [agent(0, 2), agent(1, 2)]
    try:
        # generation 1 (np=2) is training once both ranks reported ready
        kv.wait_count("/pdo/default-ej/ready/", 2, timeout=120)
        # scale out only once the 2-rank generation has checkpointed (a fixed
        # sleep raced with slow steps under a loaded pytest -n run)
        t_end = time.time() + 120
        while not list(ck.glob("ckpt-*.pt")) and time.time() < t_end:
            time.sleep(0.2)
        procs.append(agent(2, 3))
        kv.put("/paddle/default-ej/np", "3")  # what the controller's syncNP does on scale-out
        assert wait_all(procs, timeout=240) == [0, 0, 0], open(tmp_path / "e0.log").read()[-4000:]
        done = kv.get_prefix("/paddle/default-ej/done/")
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
        srv.stop()
    assert len(done) == 3
    gens = {json.loads(v)["gen"] for v in done.values()}
    assert len(gens) == 1
    readies = [r for i in range(3) for r in records(tmp_path / f"e{i}.log", "PDO_READY")]
    worlds = sorted({r["world"] for r in readies})
    assert worlds == [2, 3]
    # the 3-rank generation resumed from a checkpoint written by the 2-rank one
    assert max(r["resume_step"] for r in readies if r["world"] == 3) >= 5


def test_heter_ps_mode(tmp_path):
    """spec.heter: CPU trainers keep the sparse side, the heter worker owns the dense tower."""
    base = free_port_block()
    common = {"PADDLE_PSERVERS_IP_PORT_LIST": f"127.0.0.1:{base}",
              "PADDLE_TRAINER_ENDPOINTS": f"127.0.0.1:{base + 20},127.0.0.1:{base + 40}",
              "PADDLE_HETER_ENDPOINTS": f"127.0.0.1:{base + 60}", "PADDLE_TRAINERS_NUM": 2}
    args = ["--workload", "wide_deep", "--tiny", "--steps", "60", "--batch", "256"]
    procs = [launch(dict(common, TRAINING_ROLE="PSERVER", PADDLE_TRAINER_ID=0), args, tmp_path / "ps0.log"),
             launch(dict(common, TRAINING_ROLE="HETER", PADDLE_TRAINER_ID=0), args, tmp_path / "h0.log")]
    procs += [launch(dict(common, TRAINING_ROLE="TRAINER", PADDLE_TRAINER_ID=i), args, tmp_path / f"t{i}.log")
              for i in range(2)]
    assert wait_all(procs) == [0, 0, 0, 0], open(tmp_path / "t0.log").read()[-3000:]
    for i in range(2):
        d = records(tmp_path / f"t{i}.log", "PDO_DONE")[0]
        assert d["last_loss"] < d["first_loss"] - 0.05, d
        assert d["heter_stats"][0]["heter_steps"] >= 60  # this trainer's steps (at least) ran on the heter worker


_STORE_JOB = r"""
import os, sys, time
sys.path.insert(0, sys.argv[1])
import torch, torch.distributed as dist
from paddle_operator_amd.launch import bootstrap
b = bootstrap.init(time.time(), backend="gloo", timeout_s=60)
t = torch.ones(1) * (b.rank + 1)
dist.all_reduce(t)
assert t.item() == 3.0, t
dist.barrier()
dist.destroy_process_group()
"""


def test_concurrent_jobs_same_store_port_distinct_pod_ips():
    """Two 2-rank jobs whose rank 0s share MASTER_PORT on different loopback pod
    IPs (the local backend's exec agent): rank 0's store binds its own address
    (bootstrap._bound_store), so neither job fails with EADDRINUSE."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for ip in ("127.0.0.21", "127.0.0.22"):
        for rank in (0, 1):
            env = dict(os.environ, MASTER_ADDR=ip, MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                       LOCAL_RANK="0", OMP_NUM_THREADS="1", PDO_PIN_CPUS="0")
            procs.append(subprocess.Popen([sys.executable, "-c", _STORE_JOB, root], env=env,
                                          stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n---\n".join(outs)
