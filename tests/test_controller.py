"""Control plane (native ``_pdo_core``) on CPU.

Mirrors the reference's only behavioural test — the envtest spec
controllers/paddlejob_controller_test.go:32-113 (wide-and-deep, Service
mode, PS 3 / worker 2 → status refs 3/2, mode PS; update to PS 1 / worker 4
→ refs 1/4) — and then covers what envtest never exercised
(controllers/suite_test.go:73-77 runs without Volcano, etcd, init image or
exec): builders' env contract, ConfigMap endpoint table, Host mode ports,
Volcano gang, clean-pod policies, finalizer, failure, elastic ``np`` sync,
compat-mode sequencing, the REST apiserver and the exec agent running real
pdo-launch ranks.
"""
import json
import os
import socket
import sys
import time
import urllib.request

import pytest

from paddle_operator_amd.api import types as T

core_mod = pytest.importorskip("paddle_operator_amd._pdo_core")
from paddle_operator_amd.controller import LocalCluster  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POD = {"spec": {"containers": [{"name": "paddle", "image": "demo:v1"}]}}
POD_NEVER = {"spec": {"restartPolicy": "Never", "containers": [{"name": "paddle", "image": "demo:v1"}]}}


def refs(cl, name, role):
    st = (cl.job(name) or {}).get("status") or {}
    return len((st.get(role) or {}).get("refs") or [])


def env_of(pod):
    out = {}
    for e in pod["spec"]["containers"][0].get("env", []):
        out[e["name"]] = e.get("value", e.get("valueFrom"))
    return out


@pytest.fixture(params=["fast", "compat"])
def sim(request):
    cl = LocalCluster(mode=request.param, agent="sim", virtual_clock=True)
    yield cl
    cl.stop()


# ----------------------------------------------------------------------------- reference envtest spec
def test_reference_envtest_wide_and_deep_service(sim):
    job = T.paddlejob("wide-and-deep-service", clean_pod_policy="Never", intranet="Service",
                      ps={"replicas": 3, "template": POD_NEVER}, worker={"replicas": 2, "template": POD_NEVER})
    sim.create(job)
    assert sim.wait(lambda: refs(sim, "wide-and-deep-service", "ps") == 3 and
                    refs(sim, "wide-and-deep-service", "worker") == 2, timeout=10)
    j = sim.job("wide-and-deep-service")
    assert j["status"]["mode"] == T.Mode.PS
    j["spec"]["ps"]["replicas"] = 1
    j["spec"]["worker"]["replicas"] = 4
    sim.update(j)
    assert sim.wait(lambda: refs(sim, "wide-and-deep-service", "ps") == 1 and
                    refs(sim, "wide-and-deep-service", "worker") == 4, timeout=10)
    names = sorted(p["metadata"]["name"] for p in sim.pods("wide-and-deep-service"))
    assert names == ["wide-and-deep-service-ps-0"] + [f"wide-and-deep-service-worker-{i}" for i in range(4)]
    # one Service per pod, named like the pod; Service-mode endpoints use pod names
    assert sim.get("Service", "wide-and-deep-service-worker-3") is not None
    w0 = sim.get("Pod", "wide-and-deep-service-worker-0")
    assert env_of(w0)["POD_IP"] == "wide-and-deep-service-worker-0"
    assert w0["spec"]["containers"][0]["ports"] == [{"containerPort": 2379}]
    svcs = {s["metadata"]["name"] for s in sim.list("Service", "default")}
    if sim.opts["mode"] == "fast":  # fast mode also drops Services of scaled-in pods
        assert "wide-and-deep-service-ps-2" not in svcs
    else:  # reference behaviour: they stay until cleanup
        assert "wide-and-deep-service-ps-2" in svcs


# ----------------------------------------------------------------------------- builders
def test_pod_builder_env_contract():
    c = core_mod
    job = T.paddlejob("pj", ps={"replicas": 2, "template": POD}, worker={"replicas": 3, "template": POD})
    pod = c.construct_pod(job, "worker", 1)
    md = pod["metadata"]
    assert md["name"] == "pj-worker-1"
    assert md["labels"][T.LABEL_RESOURCE_NAME] == "pj-worker-1" and md["labels"][T.LABEL_RESOURCE_TYPE] == "worker"
    assert md["annotations"][T.ANNOTATION_RESOURCE] == "worker"
    assert pod["spec"]["hostname"] == "pj-worker-1" and pod["spec"]["subdomain"] == "pj-worker-1"
    env = env_of(pod)
    assert env["POD_IP"] == {"fieldRef": {"fieldPath": "status.podIP"}}
    assert env["PADDLE_TRAINER_ID"] == "1"
    assert env["TRAINING_ROLE"] == env["PADDLE_TRAINING_ROLE"] == "TRAINER"
    assert pod["spec"]["containers"][0]["envFrom"] == [{"configMapRef": {"name": "pj"}}]
    assert pod["spec"]["restartPolicy"] == "Never"
    assert env_of(c.construct_pod(job, "ps", 0))["TRAINING_ROLE"] == "PSERVER"
    # name/index parsing (paddlejob_helper.go:206-213)
    assert c.extract_name_index("pj-worker-12") == ("worker", 12)
    assert c.res_name("pj", "ps", 3) == "pj-ps-3"


def test_configmap_endpoint_table():
    c = core_mod
    job = T.paddlejob("pj", ps={"replicas": 2, "template": POD}, worker={"replicas": 2, "template": POD},
                      with_gloo=1)
    pods = []
    for role, n in (("ps", 2), ("worker", 2)):
        for i in range(n):
            p = c.construct_pod(job, role, i)
            p["status"] = {"podIP": f"10.0.{0 if role == 'ps' else 1}.{i + 1}"}
            pods.append(p)
    cm = c.construct_configmap(job, pods)
    d = cm["data"]
    assert d["TRAINER_PORTS_NUM"] == "20" and d["PADDLE_PORT"] == "2379"
    assert d["PADDLE_PSERVERS_IP_PORT_LIST"] == "10.0.0.1:2379,10.0.0.2:2379"
    assert d["PADDLE_TRAINER_ENDPOINTS"] == "10.0.1.1:2379,10.0.1.2:2379"
    assert d["PADDLE_TRAINERS"] == "10.0.1.1,10.0.1.2" and d["PADDLE_TRAINERS_NUM"] == "2"
    assert d["PADDLE_WITH_GLOO"] == "1" and d["PADDLE_GLOO_RENDEZVOUS"] == "3"
    assert d["PADDLE_GLOO_HTTP_ENDPOINT"] == "10.0.0.1:2397"
    # not all pods have an IPv4 yet → no ConfigMap (D-16)
    pods[-1]["status"] = {}
    assert c.construct_configmap(job, pods) is None


def test_elastic_pod_env_and_restart_policy():
    job = T.paddlejob("el", worker={"replicas": 4, "template": POD}, elastic=1)
    pod = core_mod.construct_pod(job, "worker", 0, {"etcd_endpoints": ["10.1.1.1:2379"]})
    env = env_of(pod)
    assert env["PADDLE_ELASTIC_JOB_ID"] == "default-el" and env["PADDLE_ELASTIC_NP"] == "4"
    assert env["PADDLE_ELASTIC_TIMEOUT"] == "60"
    assert pod["spec"]["restartPolicy"] == "OnFailure"
    assert "envFrom" not in pod["spec"]["containers"][0]


def test_podgroup_min_resources():
    # requests win over limits per container (paddlejob_helper.go:538-545)
    res = {"limits": {T.AMD_GPU: 8, "cpu": "4"}, "requests": {"cpu": "4", "memory": "8Gi", T.AMD_GPU: 8}}
    tmpl = {"spec": {"containers": [{"name": "c", "image": "x", "resources": res}]}}
    job = T.paddlejob("g", worker={"replicas": 2, "template": tmpl}, ps={"replicas": 1, "template": POD},
                      scheduling_policy={"minAvailable": 3, "queue": "q1", "priorityClass": "high"})
    pg = core_mod.construct_podgroup(job)
    assert pg["spec"]["minMember"] == 3 and pg["spec"]["queue"] == "q1"
    assert pg["spec"]["priorityClassName"] == "high"
    mr = pg["spec"]["minResources"]
    assert mr[T.AMD_GPU] in (16, "16") and mr["cpu"] in ("8", 8) and mr["memory"] == "16Gi"


def test_quantity_sum():
    assert core_mod.quantity_sum(["500m", "1", "1.5"]) == "3"
    assert core_mod.quantity_sum(["1Gi", "512Mi"]) == "1536Mi"


def test_phase_fsm_fixed_order():
    """D-1 fix: fixed ps→worker→heter order, Failed > Starting > Pending priority."""
    job = T.paddlejob("p", ps={"replicas": 1, "template": POD}, worker={"replicas": 2, "template": POD})
    job["status"] = {"ps": {"running": 1}, "worker": {"failed": 1, "pending": 1}}
    assert core_mod.derive_phase(job) == T.Phase.Failed
    job["status"] = {"ps": {"pending": 1}, "worker": {"running": 2}}
    assert core_mod.derive_phase(job) == T.Phase.Pending
    job["status"] = {"ps": {"running": 1}, "worker": {"running": 2}}
    assert core_mod.derive_phase(job) == T.Phase.Running
    # mixed running/succeeded keeps the previous phase (paddlejob_helper.go:120-131)
    job["status"] = {"phase": "Running", "ps": {"running": 1}, "worker": {"succeeded": 2}}
    assert core_mod.derive_phase(job) == T.Phase.Running
    job["status"] = {"phase": "Running", "ps": {"succeeded": 1}, "worker": {"succeeded": 2}}
    assert core_mod.derive_phase(job) == T.Phase.Completed
    job["status"]["phase"] = "Failed"  # terminal phases are sticky
    assert core_mod.derive_phase(job) == T.Phase.Failed
    assert core_mod.derive_mode(job) == T.Mode.PS


# ----------------------------------------------------------------------------- lifecycle
def test_collective_hostnetwork_volcano_lifecycle():
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True, volcano=True, port_range=(40000, 40100),
                      nodes=[{"name": "n0", "gpus": 8}])
    job = T.paddlejob("coll", worker={"replicas": 2, "template": POD}, intranet="Host",
                      scheduling_policy={"minAvailable": 2, "queue": "default"})
    cl.create(job)
    assert cl.wait_phase("coll", T.Phase.Running, timeout=10)
    j = cl.job("coll")
    assert T.FINALIZER in j["metadata"]["finalizers"]
    port = int(j["metadata"]["annotations"][T.ANNOTATION_HOST_PORT])
    assert 40000 <= port < 40100
    cm = cl.get("ConfigMap", "coll")["data"]
    assert cm["PADDLE_PORT"] == str(port)
    # fast mode fixes D-5: Host-mode endpoints carry the allocated port, not :2379
    assert all(ep.endswith(f":{port}") for ep in cm["PADDLE_TRAINER_ENDPOINTS"].split(","))
    p = cl.get("Pod", "coll-worker-1")
    assert p["spec"]["hostNetwork"] is True and p["spec"]["schedulerName"] == "volcano"
    pg = cl.get("PodGroup", "coll")
    assert pg["spec"]["minMember"] == 2 and pg["status"]["phase"] in ("Inqueue", "Running")
    for n in ("coll-worker-0", "coll-worker-1"):
        cl.sim_exit(n, 0)
    assert cl.wait_phase("coll", T.Phase.Completed, timeout=10)
    # default clean policy cleans pods on completion; PodGroup removed on terminal phase
    assert cl.wait(lambda: not cl.pods("coll") and cl.get("PodGroup", "coll") is None, timeout=10)
    st = cl.job("coll")["status"]
    assert st["completionTime"] and st["startTime"]
    cl.delete(T.KIND, "coll")
    assert cl.wait(lambda: cl.job("coll") is None, timeout=10)  # finalizer released the port and let go
    assert cl._c.host_ports() == 0
    cl.stop()


@pytest.mark.parametrize("policy,expect_pods", [("OnFailure", 0), ("Never", 2), ("OnCompletion", 2),
                                                ("Always", 0)])
def test_failure_and_clean_policy(policy, expect_pods):
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True)
    cl.create(T.paddlejob("f", worker={"replicas": 2, "template": POD}, clean_pod_policy=policy))
    assert cl.wait_phase("f", T.Phase.Running, timeout=10)
    cl.sim_exit("f-worker-1", 3)
    assert cl.wait_phase("f", T.Phase.Failed, timeout=10)
    cl.run_for(1.0)
    assert len(cl.pods("f")) == expect_pods
    st = cl.job("f")["status"]
    assert st["phase"] == T.Phase.Failed  # sticky even after the pods are gone
    if expect_pods:
        assert st["worker"]["failed"] == 1
    cl.stop()


def test_delete_job_with_finalizer_removes_children(sim):
    sim.create(T.paddlejob("d", ps={"replicas": 1, "template": POD}, worker={"replicas": 2, "template": POD}))
    assert sim.wait_phase("d", T.Phase.Running, timeout=10)
    sim.delete(T.KIND, "d")
    assert sim.wait(lambda: sim.job("d") is None, timeout=10)
    assert sim.wait(lambda: not sim.pods("d") and sim.get("ConfigMap", "d") is None, timeout=10)


def test_deleted_pod_is_recreated(sim):
    sim.create(T.paddlejob("r", worker={"replicas": 2, "template": POD}))
    assert sim.wait_phase("r", T.Phase.Running, timeout=10)
    uid = sim.get("Pod", "r-worker-1")["metadata"]["uid"]
    sim.delete("Pod", "r-worker-1")
    assert sim.wait(lambda: (sim.get("Pod", "r-worker-1") or {}).get("metadata", {}).get("uid") not in (None, uid),
                    timeout=10)


def test_elastic_np_sync():
    """controllers/paddlejob_elastic.go:27-55: never creates np; updates it on scale + Event Scaled."""
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True, elastic_kv=True)
    cl.create(T.paddlejob("el", worker={"replicas": 2, "template": POD}, elastic=1))
    assert cl.wait_phase("el", T.Phase.Running, timeout=10)
    assert cl.get("ConfigMap", "el") is None  # elastic jobs get no endpoint table
    assert cl.kv_get("/paddle/default-el/np") is None
    cl.scale("el", "worker", 3)
    cl.run_for(1.0)
    assert cl.kv_get("/paddle/default-el/np") is None
    cl.kv_put("/paddle/default-el/np", "3")  # the launcher's agent owns creation
    cl.scale("el", "worker", 4)
    assert cl.wait(lambda: cl.kv_get("/paddle/default-el/np") == "4", timeout=10)
    assert any(e["reason"] == "Scaled" for e in cl.events())
    assert cl.wait(lambda: len(cl.pods("el")) == 4, timeout=10)
    assert env_of(cl.get("Pod", "el-worker-3"))["PADDLE_ELASTIC_NP"] == "4"
    cl.stop()


def test_compat_mode_is_one_mutation_per_pass():
    """compat reproduces the reference's one-object-per-reconcile creation (D-3)."""
    job = T.paddlejob("c", worker={"replicas": 4, "template": POD})
    out = {}
    for mode in ("compat", "fast"):
        cl = LocalCluster(mode=mode, agent="sim", virtual_clock=True, workers=1)
        cl.create(job)
        n_pass = 0
        while len(cl.pods("c")) < 4 and n_pass < 50:
            cl.reconcile("c")
            n_pass += 1
        out[mode] = n_pass
        cl.stop()
    assert out["fast"] == 1 or out["fast"] < out["compat"]
    assert out["compat"] >= 4


def test_gpu_gang_and_device_assignment():
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True, nodes=[{"name": "n0", "gpus": 8}])
    tmpl = {"spec": {"containers": [{"name": "c", "image": "x", "resources": {"limits": {T.AMD_GPU: 2}}}]}}
    cl.create(T.paddlejob("g", worker={"replicas": 3, "template": tmpl}))
    assert cl.wait_phase("g", T.Phase.Running, timeout=10)
    assert cl.free_gpus() == {"n0": 2}
    cl.create(T.paddlejob("h", worker={"replicas": 2, "template": tmpl}))  # needs 4, only 2 free
    cl.run_for(1.0)
    assert cl.job("h")["status"].get("phase") in (None, T.Phase.Pending, "")
    cl.delete(T.KIND, "g")
    assert cl.wait_phase("h", T.Phase.Running, timeout=10)
    cl.stop()


# ----------------------------------------------------------------------------- REST apiserver
def _http(method, url, body=None):
    data = json.dumps(body).encode() if body is not None else None
    req = urllib.request.Request(url, data=data, method=method, headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return r.status, json.loads(r.read() or b"{}")
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read() or b"{}")


def test_rest_apiserver_crud():
    cl = LocalCluster(mode="fast", agent="sim")
    url = cl.serve("127.0.0.1:0")
    cl.start()
    try:
        base = f"{url}/apis/{T.GROUP}/{T.VERSION}/namespaces/default/paddlejobs"
        st, obj = _http("POST", base, T.paddlejob("rest", worker={"replicas": 2, "template": POD}))
        assert st == 201, obj
        st, _ = _http("POST", base, T.paddlejob("rest", worker={"replicas": 2, "template": POD}))
        assert st == 409
        t_end = time.time() + 10
        while time.time() < t_end:
            st, obj = _http("GET", f"{base}/rest")
            if (obj.get("status") or {}).get("phase") == "Running":
                break
            time.sleep(0.05)
        assert obj["status"]["phase"] == "Running"
        st, lst = _http("GET", f"{url}/api/v1/namespaces/default/pods?labelSelector={T.LABEL_RESOURCE_TYPE}%3Dworker")
        assert st == 200 and len(lst["items"]) == 2
        st, _ = _http("DELETE", f"{base}/rest")
        assert st == 200
        t_end = time.time() + 10
        while time.time() < t_end and _http("GET", f"{base}/rest")[0] != 404:
            time.sleep(0.05)
        assert _http("GET", f"{base}/rest")[0] == 404
        with urllib.request.urlopen(f"{url}/metrics", timeout=5) as r:
            assert b"pdo_reconcile" in r.read()
    finally:
        cl.stop()


# ----------------------------------------------------------------------------- exec agent e2e
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launcher_container(args):
    return {"name": "paddle", "image": "pdo/launcher:rocm",
            "command": [sys.executable, "-m", "paddle_operator_amd.launch"] + args,
            "env": [{"name": "PYTHONPATH", "value": REPO}, {"name": "OMP_NUM_THREADS", "value": "2"},
                    {"name": "PDO_OPS", "value": "torch"}]}


def test_exec_agent_collective_job_completes(tmp_path):
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path))
    tmpl = {"spec": {"containers": [_launcher_container(["--workload", "resnet50", "--tiny", "--steps", "3"])]}}
    cl.create(T.paddlejob("e2e", worker={"replicas": 2, "template": tmpl}, clean_pod_policy="Never"))
    try:
        ok = cl.wait_phase("e2e", T.Phase.Completed, timeout=180)
        logs = {i: open(os.path.join(cl.sandbox(f"e2e-worker-{i}"), "paddle.log")).read()
                for i in range(2) if cl.sandbox(f"e2e-worker-{i}")}
        assert ok, (cl.job("e2e")["status"], logs)
        assert len(logs) == 2
        for i, text in logs.items():
            ready = [json.loads(l[10:]) for l in text.splitlines() if l.startswith("PDO_READY ")]
            assert ready and ready[0]["rank"] == i and ready[0]["world"] == 2
    finally:
        cl.stop()


def test_exec_agent_elastic_scale_out(tmp_path):
    """Config 5 shape (elastic 2 → 3) end to end: controller np sync → agents re-rendezvous."""
    port = _free_port()
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), elastic_kv=True,
                      kv_endpoint=f"127.0.0.1:{port}")
    cl.serve(f"127.0.0.1:{port}")
    args = ["--workload", "resnet50", "--tiny", "--steps", "40", "--throttle-ms", "80",
            "--ckpt-dir", str(tmp_path / "ckpt"), "--ckpt-every", "5"]
    cont = _launcher_container(args)
    cont["env"].append({"name": "PDO_ELASTIC_TTL", "value": "3"})
    cl.create(T.paddlejob("ej", worker={"replicas": 2, "template": {"spec": {"containers": [cont]}}}, elastic=1,
                          clean_pod_policy="Never"))
    try:
        assert cl.wait(lambda: cl.kv_get("/pdo/default-ej/ready/1") is not None, timeout=120)
        cl.scale("ej", "worker", 3)
        ok = cl.wait_phase("ej", T.Phase.Completed, timeout=180)
        logs = [open(os.path.join(cl.sandbox(f"ej-worker-{i}"), "paddle.log")).read() for i in range(3)
                if cl.sandbox(f"ej-worker-{i}")]
        assert ok, (cl.job("ej")["status"], [l[-2000:] for l in logs])
        assert cl.kv_get("/paddle/default-ej/np") == "3"
        worlds = {json.loads(l[10:])["world"] for t in logs for l in t.splitlines() if l.startswith("PDO_READY ")}
        assert worlds == {2, 3}
    finally:
        cl.stop()


def _ready_rec(cl, job, rank):
    v = cl.kv_get(f"/pdo/default-{job}/ready/{rank}")
    return json.loads(v) if v else None


def test_exec_agent_elastic_scale_kill_scale_in(tmp_path):
    """Config 5 in full (scaled to CPU): elastic 2 → 3, pod kill of a rank
    (agent restarts it in place, OnFailure), scale-in 3 → 2 (controller deletes
    the surplus pod, paddlejob_controller.go:161-168), job completes.

    Each re-formed world resumes from the newest checkpoint."""
    port = _free_port()
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), elastic_kv=True,
                      kv_endpoint=f"127.0.0.1:{port}")
    cl.serve(f"127.0.0.1:{port}")
    args = ["--workload", "resnet50", "--tiny", "--steps", "90", "--throttle-ms", "60",
            "--ckpt-dir", str(tmp_path / "ckpt"), "--ckpt-every", "5"]
    cont = _launcher_container(args)
    cont["env"].append({"name": "PDO_ELASTIC_TTL", "value": "2"})
    cl.create(T.paddlejob("ek", worker={"replicas": 2, "template": {"spec": {"containers": [cont]}}}, elastic=1,
                          clean_pod_policy="Never"))

    def log(i):
        d = cl.sandbox(f"ek-worker-{i}")
        p = os.path.join(d, "paddle.log") if d else ""
        return open(p).read() if p and os.path.exists(p) else ""

    try:
        assert cl.wait(lambda: _ready_rec(cl, "ek", 1) is not None, timeout=120)
        assert cl.wait(lambda: list((tmp_path / "ckpt").glob("ckpt-*.pt")), timeout=120)
        cl.scale("ek", "worker", 3)
        def world3():  # every rank of one 3-rank generation reported ready
            recs = [_ready_rec(cl, "ek", r) or {} for r in range(3)]
            return recs[0]["gen"] if all(r.get("world") == 3 for r in recs) and \
                len({r.get("gen") for r in recs}) == 1 else None

        assert cl.wait(lambda: world3() is not None, timeout=120), log(0)[-3000:]
        gen_before = world3()
        # pod kill: SIGKILL to worker-1's process group (agent + its worker)
        assert cl.kill("ek-worker-1", 9)
        assert cl.wait(lambda: world3() not in (None, gen_before), timeout=150), log(0)[-3000:]
        pod1 = cl.get("Pod", "ek-worker-1")
        assert pod1["status"]["containerStatuses"][0]["restartCount"] >= 1
        # scale-in: np 3 → 2, the controller deletes ek-worker-2
        cl.scale("ek", "worker", 2)
        ok = cl.wait_phase("ek", T.Phase.Completed, timeout=240)
        assert ok, (cl.job("ek")["status"], log(0)[-3000:], log(1)[-3000:])
        assert cl.kv_get("/paddle/default-ek/np") == "2"
        assert cl.get("Pod", "ek-worker-2") is None
        readies = [json.loads(l[10:]) for i in range(2) for l in log(i).splitlines()
                   if l.startswith("PDO_READY ")]
        worlds = [r["world"] for r in readies if r["rank"] == 0]
        # 2-rank, 3-rank, 3-rank again after the kill, 2-rank after scale-in
        assert worlds[0] == 2 and worlds[-1] == 2 and worlds.count(3) >= 2, worlds
        assert readies[-1]["resume_step"] >= 5
    finally:
        cl.stop()


def test_exec_agent_elastic_nproc_per_pod_2(tmp_path):
    """Elastic jobs in the xGMI layout: pods of 2 local ranks each (the
    one-pod-per-node layout, --nproc-per-pod N).  np counts pods; each
    generation is a world of np × 2 ranks, forked fresh by every pod's agent.
    Scale 2 → 3 pods (world 4 → 6), kill a pod (its agent and both of its
    ranks; OnFailure restarts it in place), scale back to 2 (world 4); every
    re-formed world resumes from the newest checkpoint."""
    port = _free_port()
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), elastic_kv=True,
                      kv_endpoint=f"127.0.0.1:{port}")
    cl.serve(f"127.0.0.1:{port}")
    args = ["--workload", "resnet50", "--tiny", "--steps", "90", "--throttle-ms", "60", "--nproc-per-pod", "2",
            "--ckpt-dir", str(tmp_path / "ckpt"), "--ckpt-every", "5"]
    cont = _launcher_container(args)
    cont["env"] = [e for e in cont["env"] if e["name"] != "OMP_NUM_THREADS"] + [
        {"name": "OMP_NUM_THREADS", "value": "1"}, {"name": "PDO_ELASTIC_TTL", "value": "2"}]
    cl.create(T.paddlejob("en", worker={"replicas": 2, "template": {"spec": {"containers": [cont]}}}, elastic=1,
                          clean_pod_policy="Never"))

    def log(i):
        d = cl.sandbox(f"en-worker-{i}")
        p = os.path.join(d, "paddle.log") if d else ""
        return open(p).read() if p and os.path.exists(p) else ""

    def world(n):  # every rank of one n-rank generation reported ready → its gen
        recs = [_ready_rec(cl, "en", r) or {} for r in range(n)]
        return recs[0]["gen"] if all(r.get("world") == n for r in recs) and \
            len({r.get("gen") for r in recs}) == 1 else None

    try:
        assert cl.wait(lambda: world(4) is not None, timeout=150), log(0)[-3000:]
        assert cl.wait(lambda: list((tmp_path / "ckpt").glob("ckpt-*.pt")), timeout=120)
        cl.scale("en", "worker", 3)
        assert cl.wait(lambda: world(6) is not None, timeout=150), log(0)[-3000:]
        gen_before = world(6)
        # the scaled-in generation's ranks: pod p holds global ranks 2p, 2p + 1
        recs = [_ready_rec(cl, "en", r) for r in range(6)]
        assert [r["local_rank"] for r in recs] == [0, 1] * 3, recs
        # pod kill: SIGKILL to en-worker-1's process group (agent + both local ranks)
        assert cl.kill("en-worker-1", 9)
        assert cl.wait(lambda: world(6) not in (None, gen_before), timeout=150), log(0)[-3000:]
        assert cl.get("Pod", "en-worker-1")["status"]["containerStatuses"][0]["restartCount"] >= 1
        cl.scale("en", "worker", 2)
        ok = cl.wait_phase("en", T.Phase.Completed, timeout=240)
        assert ok, (cl.job("en")["status"], log(0)[-3000:], log(1)[-3000:])
        assert cl.kv_get("/paddle/default-en/np") == "2"
        readies = [json.loads(l[10:]) for i in range(2) for l in log(i).splitlines()
                   if l.startswith("PDO_READY ")]
        worlds = [r["world"] for r in readies if r["rank"] == 0]
        # 4 ranks, 6, 6 again after the kill, 4 after the scale-in
        assert worlds[0] == 4 and worlds[-1] == 4 and worlds.count(6) >= 2, worlds
        assert readies[-1]["resume_step"] >= 5
        assert len({r["pid"] for r in readies if r["world"] == 4 and r["gen"] == readies[-1]["gen"]}) == 4
    finally:
        cl.stop()


def test_zygote_warm_launch_and_kill(tmp_path):
    """bin/pdo-launch forks ranks from the per-node zygote; a pod kill reaches the rank."""
    pdo_launch = os.path.join(REPO, "bin", "pdo-launch")
    if not os.path.exists(pdo_launch):
        pytest.skip("bin/pdo-launch not built")
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), zygote=True)
    t_end = time.time() + 120
    while not cl.zygotes_ready() and time.time() < t_end:
        time.sleep(0.05)
    assert cl.zygotes_ready()
    cont = _launcher_container(["--workload", "noop", "--exit-after-ready"])
    cont["command"] = [pdo_launch] + cont["command"][3:]
    cl.create(T.paddlejob("z", worker={"replicas": 2, "template": {"spec": {"containers": [cont]}}},
                          clean_pod_policy="Never"))
    try:
        assert cl.wait_phase("z", T.Phase.Completed, timeout=60), cl.job("z")["status"]
        text = open(os.path.join(cl.sandbox("z-worker-1"), "paddle.log")).read()
        ready = [json.loads(l[10:]) for l in text.splitlines() if l.startswith("PDO_READY ")]
        assert ready and ready[0]["world"] == 2
        # ready well under a cold interpreter's import-torch time
        assert ready[0]["t_ready"] - ready[0]["t_start"] < 1.0, ready
        # a long-running rank: SIGTERM on the pod is relayed through the client
        cont2 = _launcher_container(["--workload", "resnet50", "--tiny", "--steps", "100000"])
        cont2["command"] = [pdo_launch] + cont2["command"][3:]
        cl.create(T.paddlejob("zk", worker={"replicas": 1, "template": {"spec": {"containers": [cont2]}}},
                              clean_pod_policy="Never"))
        assert cl.wait_phase("zk", T.Phase.Running, timeout=60)
        time.sleep(1.0)
        assert cl.kill("zk-worker-0", 15)
        assert cl.wait_phase("zk", T.Phase.Failed, timeout=30), cl.job("zk")["status"]
    finally:
        cl.stop()


def test_zygote_gpu_warm_slot_handoff(tmp_path):
    """The zygote keeps one warm slot per node GPU; a 1-GPU rank is handed to
    it (the slot becomes the rank), a replacement slot comes up, and requests
    that must not use a slot (opt-out, elastic) take the cold fork.  On a CPU
    box the slot has nothing to warm; the hand-off protocol is the same."""
    pdo_launch = os.path.join(REPO, "bin", "pdo-launch")
    if not os.path.exists(pdo_launch):
        pytest.skip("bin/pdo-launch not built")
    port = _free_port()
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), zygote=True,
                      nodes=[{"name": "node0", "gpus": 1}], kv_endpoint=f"127.0.0.1:{port}")
    cl.serve(f"127.0.0.1:{port}")
    cl.start()

    def job(name, args, extra_env=()):
        cont = _launcher_container(args)
        cont["command"] = [pdo_launch] + cont["command"][3:]
        cont["env"] += [{"name": "PDO_KV", "value": f"127.0.0.1:{port}"}] + list(extra_env)
        cont["resources"] = {"limits": {T.AMD_GPU: 1}}
        cl.create(T.paddlejob(name, worker={"replicas": 1, "template": {"spec": {"containers": [cont]}}},
                              clean_pod_policy="Never"))

    try:
        assert cl.wait_warm(timeout=120), cl.zygote_status()
        st0 = cl.zygote_status()["node0"]
        slot_pid = st0["slots"]["0"]["pid"]
        job("w1", ["--workload", "noop", "--exit-after-ready"])
        assert cl.wait_phase("w1", T.Phase.Completed, timeout=60), cl.job("w1")["status"]
        rec = _ready_rec(cl, "w1", 0)
        assert rec["warm_slot"] is True and rec["pid"] == slot_pid, rec
        assert cl.wait_warm(timeout=120)
        st1 = cl.zygote_status()["node0"]
        assert st1["served"]["warm"] == 1 and st1["slots"]["0"]["pid"] != slot_pid
        # opted out: cold fork, the slot stays
        job("w2", ["--workload", "noop", "--exit-after-ready"], [{"name": "PDO_WARM_SLOT", "value": "0"}])
        assert cl.wait_phase("w2", T.Phase.Completed, timeout=60)
        assert _ready_rec(cl, "w2", 0)["warm_slot"] is False
        # a different runtime environment (NCCL_* read once per process): cold
        job("w3", ["--workload", "noop", "--exit-after-ready"], [{"name": "NCCL_DEBUG", "value": "WARN"}])
        assert cl.wait_phase("w3", T.Phase.Completed, timeout=60)
        assert _ready_rec(cl, "w3", 0)["warm_slot"] is False
        st2 = cl.zygote_status()["node0"]
        assert {k: st2["served"][k] for k in ("warm", "cold")} == {"warm": 1, "cold": 2}
        assert st2["slots"]["0"]["pid"] == st1["slots"]["0"]["pid"]
        # a long-running rank on a slot: the pod kill reaches it
        job("wk", ["--workload", "resnet50", "--tiny", "--steps", "100000"])
        assert cl.wait_phase("wk", T.Phase.Running, timeout=60)
        assert cl.wait(lambda: _ready_rec(cl, "wk", 0) is not None, timeout=60)
        rec = _ready_rec(cl, "wk", 0)
        assert rec["warm_slot"] is True
        assert cl.kill("wk-worker-0", 15)
        assert cl.wait_phase("wk", T.Phase.Failed, timeout=30), cl.job("wk")["status"]
        assert cl.wait(lambda: not os.path.exists(f"/proc/{rec['pid']}") or
                       open(f"/proc/{rec['pid']}/stat").read().split()[2] == "Z", timeout=10)
    finally:
        cl.stop()


def test_elastic_member_rejoins_after_lease_loss(tmp_path):
    """A member whose KV lease is gone (expired while pdo-kv was unreachable,
    here: revoked from outside) re-grants and re-announces instead of sitting
    in rendezvous until the timeout (rc=3 → pod restart); the world re-forms
    and the job completes without a restart."""
    from paddle_operator_amd.kv.client import KVClient
    port = _free_port()
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), elastic_kv=True,
                      kv_endpoint=f"127.0.0.1:{port}")
    cl.serve(f"127.0.0.1:{port}")
    args = ["--workload", "resnet50", "--tiny", "--steps", "40", "--throttle-ms", "60",
            "--ckpt-dir", str(tmp_path / "ckpt"), "--ckpt-every", "5"]
    cont = _launcher_container(args)
    cont["env"].append({"name": "PDO_ELASTIC_TTL", "value": "2"})
    cl.create(T.paddlejob("el", worker={"replicas": 2, "template": {"spec": {"containers": [cont]}}}, elastic=1,
                          clean_pod_policy="Never"))

    def log(i):
        d = cl.sandbox(f"el-worker-{i}")
        p = os.path.join(d, "paddle.log") if d else ""
        return open(p).read() if p and os.path.exists(p) else ""

    try:
        assert cl.wait(lambda: _ready_rec(cl, "el", 1) is not None, timeout=120)
        kv = KVClient(f"127.0.0.1:{port}")
        node = json.loads(kv.get("/paddle/default-el/nodes/000001"))
        kv.lease_revoke(int(node["lease"]))  # the member's record vanishes with its lease
        assert cl.wait(lambda: "re-registered" in log(1), timeout=30), log(1)[-3000:]
        node2 = json.loads(kv.get("/paddle/default-el/nodes/000001"))
        assert node2["lease"] != node["lease"]
        ok = cl.wait_phase("el", T.Phase.Completed, timeout=180)
        assert ok, (cl.job("el")["status"], log(0)[-2000:], log(1)[-2000:])
        pod1 = cl.get("Pod", "el-worker-1")
        assert pod1["status"]["containerStatuses"][0]["restartCount"] == 0
        gens = {json.loads(l[10:]).get("gen") for l in log(1).splitlines() if l.startswith("PDO_READY ")}
        assert len(gens) >= 2  # the world re-formed around the new lease
    finally:
        cl.stop()


@pytest.mark.parametrize("visibility", ["isolate", "all"])
def test_exec_agent_gpu_visibility_modes(tmp_path, monkeypatch, visibility):
    """Default: each pod sees only its GPUs (HIP_VISIBLE_DEVICES, as a device
    plugin).  PDO_GPU_VISIBILITY=all on the agent: every GPU stays visible and
    the pod's own ids come in PDO_GPU_IDS (launch/bootstrap.py selects it) — the
    torchrun-style layout bench.py uses so RCCL sees its xGMI peers as local
    devices."""
    if visibility == "all":
        monkeypatch.setenv("PDO_GPU_VISIBILITY", "all")
    else:
        monkeypatch.delenv("PDO_GPU_VISIBILITY", raising=False)
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    cl = LocalCluster(mode="fast", agent="exec", sandbox_root=str(tmp_path), nodes=[{"name": "n0", "gpus": 2}])
    c = {"name": "paddle", "image": "busybox", "command": ["sh", "-c", "env | grep -E '^(PDO_GPU_IDS|HIP_VISIBLE_DEVICES)=' | sort"],
         "resources": {"limits": {T.AMD_GPU: 1}}}
    cl.create(T.paddlejob("vis", worker={"replicas": 2, "template": {"spec": {"containers": [c]}}},
                          clean_pod_policy="Never"))
    try:
        assert cl.wait_phase("vis", T.Phase.Completed, timeout=60), cl.job("vis")["status"]
        seen = sorted(open(os.path.join(cl.sandbox(f"vis-worker-{i}"), "paddle.log")).read().strip() for i in range(2))
        key = "PDO_GPU_IDS" if visibility == "all" else "HIP_VISIBLE_DEVICES"
        assert seen == [f"{key}=0", f"{key}=1"], seen
    finally:
        cl.stop()
