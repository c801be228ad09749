"""BASELINE.json configs 1, 4 and 5 driven through the operator (CPU).

* Config 1 — wide&deep PS PaddleJob (1 pserver + 1 trainer, withGloo 1) on
  the exec agent: controller → ConfigMap ``envFrom`` → native start gate
  (ps released before the trainer, paddlejob_controller.go:318-330) →
  ``pdo-launch`` → RPC parameter server; the model learns.  Reference:
  deploy/examples/wide_and_deep.yaml:1-21, paddlejob_helper.go:215-279.
* Config 4 — GPT-2-medium collective PaddleJob, ``--scheduling=volcano``,
  ``minMember=8``, on a simulated 8-GPU node: all-or-nothing binding, PodGroup
  deleted on completion (paddlejob_controller.go:133-157).
* Config 5 — elastic 4 → 8 → 4 with a pod kill on the sim backend with GPU
  accounting (deploy/elastic/resnet.yaml:1-37; the exec-agent variant with real
  ranks is tests/test_controller.py::test_exec_agent_elastic_scale_kill_scale_in).
* The native start gate itself (sim agent): ps → worker → heter ordering with
  no coordinator container and no exec.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from paddle_operator_amd.api import types as T

pytest.importorskip("paddle_operator_amd._pdo_core")
from paddle_operator_amd.controller import LocalCluster  # noqa: E402

from test_launch import free_port_block  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POD = {"spec": {"containers": [{"name": "paddle", "image": "demo:v1"}]}}
GATE = "pdo.amd.com/start-gate"


def _running(pod):
    cs = (pod.get("status") or {}).get("containerStatuses") or []
    return bool(cs) and all("running" in (c.get("state") or {}) for c in cs)


def _role_pods(cl, job, role):
    return [p for p in cl.pods(job) if p["metadata"]["annotations"].get("paddle-resource") == role]


# ----------------------------------------------------------------------------- native start gate
def test_native_start_gate_orders_roles():
    """ps → worker → heter: no main container of a role runs before every pod
    of the earlier roles is really running; only one API write per role."""
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True, sim_start_delay=0.5)
    job = T.paddlejob("gate", ps={"replicas": 2, "template": POD}, worker={"replicas": 3, "template": POD},
                      heter={"replicas": 1, "template": POD})
    cl.create(job)
    order = ["ps", "worker", "heter"]
    seen_held = set()
    try:
        for _ in range(400):
            cl.run_for(0.02)
            pods = {r: _role_pods(cl, "gate", r) for r in order}
            for i, r in enumerate(order):
                for p in pods[r]:
                    if p["metadata"]["annotations"].get(GATE) == "hold":
                        seen_held.add(r)
                    if _running(p):  # an earlier role must be complete and running
                        for e in order[:i]:
                            assert len(pods[e]) == job["spec"][e]["replicas"] and \
                                all(_running(q) for q in pods[e]), (r, e)
            if (cl.job("gate").get("status") or {}).get("phase") == T.Phase.Running:
                break
        st = cl.job("gate")["status"]
        assert st["phase"] == T.Phase.Running, st
        assert seen_held == {"worker", "heter"}  # the first role is never held
        assert all(p["metadata"]["annotations"].get(GATE, "released") == "released" for p in cl.pods("gate"))
        assert not any(c["name"] == "coord-paddle" for p in cl.pods("gate")
                       for c in p["spec"].get("initContainers") or [])
    finally:
        cl.stop()


def test_start_gate_off_in_compat_and_for_single_role():
    for mode, job, gated in (
            ("compat", T.paddlejob("a", ps={"replicas": 1, "template": POD},
                                   worker={"replicas": 1, "template": POD}), False),
            ("fast", T.paddlejob("b", worker={"replicas": 2, "template": POD}), False)):
        cl = LocalCluster(mode=mode, agent="sim", virtual_clock=True)
        cl.create(job)
        name = job["metadata"]["name"]
        assert cl.wait_phase(name, T.Phase.Running, timeout=20)
        assert any(GATE in p["metadata"]["annotations"] for p in cl.pods(name)) == gated
        cl.stop()


def test_recreated_pod_of_released_role_is_released_again():
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True)
    cl.create(T.paddlejob("rg", ps={"replicas": 1, "template": POD}, worker={"replicas": 2, "template": POD}))
    try:
        assert cl.wait_phase("rg", T.Phase.Running, timeout=10)
        uid = cl.get("Pod", "rg-worker-1")["metadata"]["uid"]
        cl.delete("Pod", "rg-worker-1")
        assert cl.wait(lambda: (cl.get("Pod", "rg-worker-1") or {}).get("metadata", {}).get("uid") not in (None, uid)
                       and _running(cl.get("Pod", "rg-worker-1")), timeout=10)
        assert cl.get("Pod", "rg-worker-1")["metadata"]["annotations"][GATE] == "released"
    finally:
        cl.stop()


# ----------------------------------------------------------------------------- config 1
def test_config1_wide_deep_ps_job_through_operator(tmp_path):
    """1 pserver + 1 trainer, withGloo 1, on the exec agent (real pdo-launch ranks)."""
    base = free_port_block(30)
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), port_range=(base, base + 20))
    cont = {"name": "paddle", "image": "pdo/launcher:rocm",
            "command": [sys.executable, "-m", "paddle_operator_amd.launch", "--workload", "wide_deep", "--tiny",
                        "--steps", "60", "--batch", "256"],
            "env": [{"name": "PYTHONPATH", "value": REPO}, {"name": "OMP_NUM_THREADS", "value": "2"},
                    {"name": "PDO_OPS", "value": "torch"}]}
    tmpl = {"spec": {"containers": [cont]}}
    # Host intranet: one allocated port block per job, so concurrently running
    # tests never share :2379 on the node's loopback address
    cl.create(T.paddlejob("wide-ande-deep", ps={"replicas": 1, "template": tmpl},
                          worker={"replicas": 1, "template": tmpl}, with_gloo=1, intranet="Host",
                          clean_pod_policy="Never"))

    def log(pod):
        d = cl.sandbox(pod)
        p = os.path.join(d, "paddle.log") if d else ""
        return open(p).read() if p and os.path.exists(p) else ""

    def recs(pod, tag):
        return [json.loads(l[len(tag) + 1:]) for l in log(pod).splitlines() if l.startswith(tag + " ")]

    try:
        ok = cl.wait_phase("wide-ande-deep", T.Phase.Completed, timeout=240)
        assert ok, (cl.job("wide-ande-deep")["status"], log("wide-ande-deep-ps-0")[-3000:],
                    log("wide-ande-deep-worker-0")[-3000:])
        cm = cl.get("ConfigMap", "wide-ande-deep")["data"]
        assert cm["PADDLE_WITH_GLOO"] == "1" and cm["PADDLE_TRAINERS_NUM"] == "1"
        assert cm["PADDLE_PSERVERS_IP_PORT_LIST"].count(",") == 0
        ps_ready = recs("wide-ande-deep-ps-0", "PDO_READY")[0]
        tr_ready = recs("wide-ande-deep-worker-0", "PDO_READY")[0]
        assert ps_ready["role"] == "PSERVER" and tr_ready["role"] == "TRAINER"
        assert ps_ready["backend"] == "rpc+gloo"
        # the trainer's container was started only once the pserver's ran (native gate)
        ps = cl.get("Pod", "wide-ande-deep-ps-0")
        trainer = cl.get("Pod", "wide-ande-deep-worker-0")
        assert trainer["metadata"]["annotations"][GATE] == "released" and GATE not in ps["metadata"]["annotations"]
        started = lambda p: p["status"]["containerStatuses"][0]["state"]["terminated"]["startedAt"]  # noqa: E731
        assert started(trainer) >= started(ps)
        done = recs("wide-ande-deep-worker-0", "PDO_DONE")[0]
        assert done["last_loss"] < done["first_loss"] - 0.05, done
        st = cl.job("wide-ande-deep")["status"]
        assert st["mode"] == T.Mode.PS and st["startTime"] and st["completionTime"]
    finally:
        cl.stop()


# ----------------------------------------------------------------------------- config 4
def _gpt2_tmpl(gpus=1):
    return {"spec": {"containers": [{
        "name": "paddle", "image": "pdo/launcher:rocm",
        "command": ["pdo-launch", "--workload", "gpt2", "--model", "gpt2-medium", "--batch", "64", "--seq", "1024"],
        "resources": {"limits": {T.AMD_GPU: gpus}}}]}}


def test_config4_gpt2_volcano_gang_min_member_8():
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True, volcano=True,
                      nodes=[{"name": "mi355x-0", "gpus": 8}])
    try:
        # another job holds one GPU: the 8-rank gang must not bind partially
        cl.create(T.paddlejob("other", worker={"replicas": 1, "template": _gpt2_tmpl()}))
        assert cl.wait_phase("other", T.Phase.Running, timeout=10)
        cl.create(T.paddlejob("gpt2m", worker={"replicas": 8, "template": _gpt2_tmpl()},
                              scheduling_policy={"minAvailable": 8, "queue": "default"}))
        cl.run_for(2.0)
        pg = cl.get("PodGroup", "gpt2m")
        assert pg["spec"]["minMember"] == 8
        assert pg["spec"]["minResources"][T.AMD_GPU] in ("8", 8)
        assert (pg.get("status") or {}).get("phase", "Pending") == "Pending"
        assert not any(p["spec"].get("nodeName") for p in cl.pods("gpt2m"))  # nothing bound
        assert cl.free_gpus() == {"mi355x-0": 7}
        # the GPU frees up → the whole gang binds at once
        cl.sim_exit("other-worker-0", 0)
        assert cl.wait_phase("gpt2m", T.Phase.Running, timeout=20), cl.job("gpt2m")["status"]
        pods = cl.pods("gpt2m")
        assert len(pods) == 8 and all(p["spec"]["nodeName"] == "mi355x-0" for p in pods)
        assert all(p["spec"]["schedulerName"] == "volcano" and
                   p["metadata"]["annotations"]["scheduling.k8s.io/group-name"] == "gpt2m" for p in pods)
        assert cl.free_gpus() == {"mi355x-0": 0}
        env = {e["name"]: e.get("value") for e in pods[0]["spec"]["containers"][0]["env"]}
        assert env["PDO_REPLICAS"] == "8"
        for i in range(8):
            cl.sim_exit(f"gpt2m-worker-{i}", 0)
        assert cl.wait_phase("gpt2m", T.Phase.Completed, timeout=20)
        assert cl.wait(lambda: cl.get("PodGroup", "gpt2m") is None, timeout=10)  # terminal → PG deleted
        assert cl.wait(lambda: cl.free_gpus() == {"mi355x-0": 8}, timeout=10)
    finally:
        cl.stop()


# ----------------------------------------------------------------------------- config 5
def test_config5_elastic_4_8_4_with_pod_kill_gpu_accounting():
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True, elastic_kv=True,
                      nodes=[{"name": "mi355x-0", "gpus": 8}])
    try:
        cl.create(T.paddlejob("eres", worker={"replicas": 4, "template": _gpt2_tmpl()}, elastic=1))
        assert cl.wait_phase("eres", T.Phase.Running, timeout=10)
        assert cl.free_gpus() == {"mi355x-0": 4}
        cl.kv_put("/paddle/default-eres/np", "4")  # the in-container launcher owns creation
        cl.scale("eres", "worker", 8)
        # scale-out: np first, then the pods (paddlejob_controller.go:209-219 before :277-287)
        assert cl.wait(lambda: cl.kv_get("/paddle/default-eres/np") == "8", timeout=10)
        assert cl.wait(lambda: len(cl.pods("eres")) == 8 and all(_running(p) for p in cl.pods("eres")), timeout=10)
        assert cl.free_gpus() == {"mi355x-0": 0}
        env7 = {e["name"]: e.get("value") for e in cl.get("Pod", "eres-worker-7")["spec"]["containers"][0]["env"]}
        assert env7["PADDLE_ELASTIC_NP"] == "8" and env7["PADDLE_ELASTIC_JOB_ID"] == "default-eres"
        # pod kill: OnFailure restarts in place, the GPU stays with the pod
        assert cl.get("Pod", "eres-worker-2")["spec"]["restartPolicy"] == "OnFailure"
        cl.sim_exit("eres-worker-2", 137)
        assert cl.wait(lambda: (cl.get("Pod", "eres-worker-2")["status"]["containerStatuses"][0]
                                ["restartCount"]) >= 1 and _running(cl.get("Pod", "eres-worker-2")), timeout=10)
        assert cl.free_gpus() == {"mi355x-0": 0}
        assert cl.job("eres")["status"]["phase"] == T.Phase.Running
        # scale-in: surplus pods go first, then np (controller.go:161-168 before :209-219)
        cl.scale("eres", "worker", 4)
        assert cl.wait(lambda: len(cl.pods("eres")) == 4 and cl.kv_get("/paddle/default-eres/np") == "4",
                       timeout=10)
        assert sorted(p["metadata"]["name"] for p in cl.pods("eres")) == [f"eres-worker-{i}" for i in range(4)]
        assert cl.wait(lambda: cl.free_gpus() == {"mi355x-0": 4}, timeout=10)
        assert sum(e["reason"] == "Scaled" for e in cl.events()) >= 2
    finally:
        cl.stop()


# ----------------------------------------------------------------------------- multi-GPU pods
def test_two_pods_nproc_per_pod_2_world_4(tmp_path):
    """2 replicas × --nproc-per-pod 2 through the operator: each pod's entry
    process supervises two local ranks (RANK = trainer_id·2 + local), one world
    of 4 over gloo — the layout of one pod per node holding all its GPUs
    (amd.com/gpu: 8, --nproc-per-pod 8), where RCCL reaches every peer over xGMI."""
    base = free_port_block(50)
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), port_range=(base, base + 40))
    cont = {"name": "paddle", "image": "pdo/launcher:rocm",
            "command": [sys.executable, "-m", "paddle_operator_amd.launch", "--workload", "gpt2", "--tiny",
                        "--steps", "3", "--log-every", "1", "--seq", "128", "--nproc-per-pod", "2",
                        "--backend", "gloo"],
            "env": [{"name": "PYTHONPATH", "value": REPO}, {"name": "OMP_NUM_THREADS", "value": "1"},
                    {"name": "PDO_OPS", "value": "torch"}]}
    cl.create(T.paddlejob("np2", worker={"replicas": 2, "template": {"spec": {"containers": [cont]}}},
                          intranet="Host", clean_pod_policy="Never"))

    def log(pod):
        d = cl.sandbox(pod)
        p = os.path.join(d, "paddle.log") if d else ""
        return open(p).read() if p and os.path.exists(p) else ""

    def recs(pod, tag):
        return [json.loads(l[len(tag) + 1:]) for l in log(pod).splitlines() if l.startswith(tag + " ")]

    try:
        ok = cl.wait_phase("np2", T.Phase.Completed, timeout=300)
        assert ok, (cl.job("np2")["status"], log("np2-worker-0")[-3000:], log("np2-worker-1")[-3000:])
        for i in range(2):
            ready = sorted(recs(f"np2-worker-{i}", "PDO_READY"), key=lambda r: r["rank"])
            assert [r["rank"] for r in ready] == [2 * i, 2 * i + 1], ready
            assert [r["local_rank"] for r in ready] == [0, 1]
            assert all(r["world"] == 4 and r["backend"] == "gloo" for r in ready)
            assert len({r["pid"] for r in ready}) == 2  # two processes in one pod
            done = recs(f"np2-worker-{i}", "PDO_DONE")
            assert len(done) == 2 and all(d["steps"] == 3 and d["world"] == 4 for d in done)
        st = cl.job("np2")["status"]
        assert st["mode"] == T.Mode.Collective and st["worker"]["succeeded"] == 2
    finally:
        cl.stop()


def test_nproc_per_pod_local_rank_failure_takes_pod_down(tmp_path):
    """A local rank that fails ends its siblings and fails the pod (its status
    is the pod's), so the job goes Failed instead of hanging in a collective."""
    from paddle_operator_amd.launch.env import JobEnv
    env = JobEnv.from_env({"PADDLE_TRAINER_ID": "1", "PADDLE_TRAINERS_NUM": "2",
                           "PADDLE_TRAINER_ENDPOINTS": "10.0.0.1:2379,10.0.0.2:2379"})
    assert env.torch_env(1, 4) == {"RANK": "5", "WORLD_SIZE": "8", "LOCAL_RANK": "1", "LOCAL_WORLD_SIZE": "4",
                                   "MASTER_ADDR": "10.0.0.1", "MASTER_PORT": "2380"}
    base = free_port_block(10)
    e = dict(os.environ, PYTHONPATH=REPO, PADDLE_TRAINER_ID="0", PADDLE_TRAINERS_NUM="1",
             PADDLE_TRAINER_ENDPOINTS=f"127.0.0.1:{base}", POD_IP="127.0.0.1", PADDLE_PORT=str(base),
             TRAINING_ROLE="TRAINER", PDO_OPS="torch", OMP_NUM_THREADS="1")
    # world 2 in one pod, but a bogus workload model makes every local rank fail at start
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "paddle_operator_amd.launch", "--workload", "gpt2",
                        "--model", "no-such-model", "--nproc-per-pod", "2", "--backend", "gloo", "--timeout", "60"],
                       env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0, r.stdout[-2000:]
    assert time.time() - t0 < 200
    assert "local ranks" in r.stdout
