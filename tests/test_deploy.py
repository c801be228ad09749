"""Deploy surface: generated manifests current + valid; native unit tests; license headers."""
import os
import subprocess
import sys

import pytest
import yaml

from paddle_operator_amd import deploy
from paddle_operator_amd.api import types as T

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_manifests_are_current():
    r = subprocess.run([sys.executable, "-m", "paddle_operator_amd.deploy", "--check"], cwd=REPO,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_crd_identity():
    docs = list(yaml.safe_load_all(open(os.path.join(REPO, "deploy/v1/crd.yaml"))))
    crd = docs[0]
    assert crd["metadata"]["name"] == "paddlejobs.batch.paddlepaddle.org"
    names = crd["spec"]["names"]
    assert names["kind"] == "PaddleJob" and names["shortNames"] == ["pdj"] and names["plural"] == "paddlejobs"
    v = crd["spec"]["versions"][0]
    assert v["name"] == "v1" and v["subresources"] == {"status": {}}
    assert [c["name"] for c in v["additionalPrinterColumns"]] == ["Status", "Mode", "Age"]
    props = v["schema"]["openAPIV3Schema"]["properties"]["spec"]["properties"]
    for k in ("cleanPodPolicy", "schedulingPolicy", "intranet", "withGloo", "ps", "worker", "heter", "elastic"):
        assert k in props


def test_examples_validate_and_request_amd_gpus():
    core = pytest.importorskip("paddle_operator_amd._pdo_core")
    for name, job in deploy.example_jobs().items():
        T.validate(job)
        assert core.validate(job) == [], name  # list of problems
        text = yaml.safe_dump(job)
        assert "nvidia.com/gpu" not in text
    gpt = deploy.example_jobs()["gpt2_medium_volcano.yaml"]
    assert gpt["spec"]["schedulingPolicy"]["minAvailable"] == 8
    assert gpt["spec"]["worker"]["template"]["spec"]["containers"][0]["resources"]["limits"][T.AMD_GPU] == 1
    assert deploy.example_jobs()["elastic_resnet.yaml"]["spec"]["elastic"] == 1


def test_operator_manifest_rbac_covers_controller():
    docs = list(yaml.safe_load_all(open(os.path.join(REPO, "deploy/v1/operator.yaml"))))
    kinds = [d["kind"] for d in docs]
    for k in ("Namespace", "ServiceAccount", "ClusterRole", "ClusterRoleBinding", "Deployment", "Service"):
        assert k in kinds
    role = next(d for d in docs if d["kind"] == "ClusterRole" and d["metadata"]["name"] == "pdo-manager-role")
    res = {r for rule in role["rules"] for r in rule["resources"]}
    for r in ("pods", "services", "configmaps", "events", "paddlejobs", "paddlejobs/status", "podgroups", "pods/exec"):
        assert r in res
    mgr = next(d for d in docs if d["kind"] == "Deployment" and d["metadata"]["name"] == "pdo-manager")
    args = mgr["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "--backend=k8s" in args and any(a.startswith("--etcd-server=") for a in args)


def test_helm_chart_present():
    for f in ("Chart.yaml", "values.yaml", "templates/manager.yaml", "templates/kv.yaml", "crds/paddlejob.yaml"):
        assert os.path.exists(os.path.join(REPO, "charts/pdo-operator", f)), f
    vals = yaml.safe_load(open(os.path.join(REPO, "charts/pdo-operator/values.yaml")))
    assert vals["manager"]["mode"] in ("fast", "compat")


def test_native_core_unit_tests():
    exe = os.path.join(REPO, "bin", "pdo-core-tests")
    if not os.path.exists(exe):
        pytest.skip("native tests not built")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_license_headers():
    r = subprocess.run([sys.executable, "tools/license.py"], cwd=REPO, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
