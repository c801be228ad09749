"""CRD structural schema: the reference's embedded PodTemplateSpec schema
(deploy/v1/crd.yaml:59-3146) validates role templates and prunes unknown
fields at admission — e.g. the misspelled ``cleanPolicy`` of
docs/user-guide.md:312 disappears (quirk D-9).  The native local apiserver
(csrc/core/schema.cpp) and the Python side (api/podschema.py) run the same
algorithm over the same schema."""
import copy
import json

import pytest

from paddle_operator_amd.api import crd as CRD
from paddle_operator_amd.api import podschema as PS
from paddle_operator_amd.api import types as T

core = pytest.importorskip("paddle_operator_amd._pdo_core")
from paddle_operator_amd.controller import LocalCluster  # noqa: E402

TMPL = {"metadata": {"labels": {"app": "x"}, "annotations": {"a": "b"}, "bogus": 1},
        "spec": {"containers": [{"name": "paddle", "image": "pdo/launcher:rocm", "imagee": "typo",
                                 "command": ["pdo-launch"], "env": [{"name": "A", "value": "1", "junk": True}],
                                 "resources": {"limits": {T.AMD_GPU: 1, "memory": "8Gi"}},
                                 "volumeMounts": [{"name": "shm", "mountPath": "/dev/shm"}]}],
                 "volumes": [{"name": "shm", "emptyDir": {"medium": "Memory"}},
                             {"name": "ckpt", "hostPath": {"path": "/tmp/checkpoint"}},
                             {"name": "p", "projected": {"sources": [{"anything": {"kept": 1}}]}}],
                 "nodeSelector": {"accelerator": "mi355x"}, "notAPodField": "x",
                 "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                     "nodeSelectorTerms": [{"matchExpressions": [{"key": "k", "operator": "In", "values": ["v"]}]}]}}}}}


def _job(**over):
    j = T.paddlejob("s", worker={"replicas": 2, "template": copy.deepcopy(TMPL)})
    j["spec"]["cleanPolicy"] = "Always"  # docs/user-guide.md:312 typo
    j["spec"].update(over)
    return j


def _expect_pruned(spec):
    assert "cleanPolicy" not in spec
    t = spec["worker"]["template"]
    assert "bogus" not in t["metadata"] and t["metadata"]["labels"] == {"app": "x"}
    c = t["spec"]["containers"][0]
    assert "imagee" not in c and c["image"] == "pdo/launcher:rocm"
    assert c["env"] == [{"name": "A", "value": "1"}]
    assert c["resources"]["limits"][T.AMD_GPU] in (1, "1")
    assert "notAPodField" not in t["spec"] and t["spec"]["nodeSelector"] == {"accelerator": "mi355x"}
    vols = {v["name"]: v for v in t["spec"]["volumes"]}
    assert vols["ckpt"]["hostPath"]["path"] == "/tmp/checkpoint"
    assert vols["p"]["projected"]["sources"][0]["anything"] == {"kept": 1}  # preserve-unknown leaf
    terms = t["spec"]["affinity"]["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"]
    assert terms["nodeSelectorTerms"][0]["matchExpressions"][0]["values"] == ["v"]


def test_crd_embeds_structural_pod_template_schema():
    s = CRD.openapi_schema()["properties"]["spec"]["properties"]
    for role in ("ps", "worker", "heter"):
        t = s[role]["properties"]["template"]
        assert "x-kubernetes-preserve-unknown-fields" not in t
        assert t["properties"]["spec"]["required"] == ["containers"]
        assert t["properties"]["spec"]["properties"]["containers"]["items"]["required"] == ["name"]


def test_python_prune_and_check():
    j = _job()
    pruned = PS.prune(j, CRD.openapi_schema())
    _expect_pruned(pruned["spec"])
    assert PS.check(pruned, CRD.openapi_schema()) == []
    bad = _job()
    del bad["spec"]["worker"]["template"]["spec"]["containers"][0]["name"]
    bad["spec"]["worker"]["template"]["spec"]["containers"][0]["command"] = "not-a-list"
    errs = PS.check(bad, CRD.openapi_schema())
    assert "spec.worker.template.spec.containers[0].name: Required value" in errs
    assert any(e.startswith("spec.worker.template.spec.containers[0].command: Invalid value") for e in errs)


def test_native_apiserver_prunes_on_create_and_update():
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True)
    try:
        cl.create(_job())
        stored = cl.job("s")
        _expect_pruned(stored["spec"])
        # python and native pruning agree field for field
        py = PS.prune(_job(), CRD.openapi_schema())
        assert json.dumps(py["spec"], sort_keys=True) == json.dumps(stored["spec"], sort_keys=True)
        stored["spec"]["worker"]["template"]["spec"]["containers"][0]["imagee"] = "again"
        cl.update(stored)
        assert "imagee" not in cl.job("s")["spec"]["worker"]["template"]["spec"]["containers"][0]
        assert cl.wait_phase("s", T.Phase.Running, timeout=10)
    finally:
        cl.stop()


@pytest.mark.parametrize("mutate,needle", [
    (lambda j: j["spec"]["worker"]["template"]["spec"].pop("containers"), "spec.worker.template.spec.containers"),
    (lambda j: j["spec"]["worker"].__setitem__("replicas", "two"), "spec.worker.replicas"),
    (lambda j: j["spec"]["worker"]["template"]["spec"]["containers"][0].pop("name"), "containers[0].name"),
    (lambda j: j["spec"]["worker"]["template"]["spec"]["volumes"][1]["hostPath"].pop("path"), "hostPath.path"),
])
def test_native_apiserver_rejects_invalid(mutate, needle):
    cl = LocalCluster(mode="fast", agent="sim", virtual_clock=True)
    try:
        j = _job()
        mutate(j)
        with pytest.raises(core.ApiError) as ei:
            cl.create(j)
        assert needle in str(ei.value) and "is invalid" in str(ei.value)
        assert cl.job("s") is None
    finally:
        cl.stop()


def test_examples_pass_structural_validation():
    import glob
    import os

    import yaml
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = glob.glob(os.path.join(root, "deploy", "examples", "*.yaml")) + \
        glob.glob(os.path.join(root, "deploy", "elastic", "*resnet*.yaml"))
    assert files
    for f in files:
        for doc in yaml.safe_load_all(open(f)):
            if doc and doc.get("kind") == T.KIND:
                assert PS.check(doc, CRD.openapi_schema()) == [], f
                assert PS.prune(doc, CRD.openapi_schema()) == doc, f  # nothing of ours is pruned
