"""pdo-manager binary (local backend) driven by pdoctl over its REST API."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from paddle_operator_amd.client import PaddleJobClient, main as pdoctl

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MANAGER = os.path.join(REPO, "bin", "pdo-manager")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def manager(tmp_path):
    if not os.path.exists(MANAGER):
        pytest.skip("pdo-manager not built")
    api = _port()
    proc = subprocess.Popen([MANAGER, "--backend=local", "--agent=exec", "--gpus=0", f"--api-bind-address=127.0.0.1:{api}",
                             "--metrics-bind-address=0", "--health-probe-bind-address=0",
                             f"--sandbox-root={tmp_path}/sb"], stdout=open(tmp_path / "mgr.log", "w"),
                            stderr=subprocess.STDOUT, start_new_session=True)
    url = f"http://127.0.0.1:{api}"
    c = PaddleJobClient(url)
    t_end = time.time() + 20
    while time.time() < t_end:
        try:
            c.list()
            break
        except Exception:
            time.sleep(0.05)
    yield url, c, tmp_path
    proc.terminate()
    try:
        proc.wait(10)
    except subprocess.TimeoutExpired:
        proc.kill()


def test_pdoctl_lifecycle(manager, capsys):
    url, c, tmp = manager
    job = tmp / "job.yaml"
    job.write_text(f"""
apiVersion: batch.paddlepaddle.org/v1
kind: PaddleJob
metadata:
  name: demo
spec:
  cleanPodPolicy: Never
  worker:
    replicas: 2
    template:
      spec:
        containers:
        - name: paddle
          image: x
          command: ["{sys.executable}", "-u", "-c", "import os,time; print('rank', os.environ['PADDLE_TRAINER_ID'], os.environ.get('PADDLE_TRAINERS_NUM')); time.sleep(30)"]
""")
    assert pdoctl(["--server", url, "apply", "-f", str(job)]) == 0
    assert pdoctl(["--server", url, "wait", "demo", "--phase", "Running", "--timeout", "30"]) == 0
    capsys.readouterr()
    assert pdoctl(["--server", url, "get"]) == 0
    out = capsys.readouterr().out
    assert "demo" in out and "Running" in out and "Collective" in out
    assert pdoctl(["--server", url, "get", "demo", "-o", "json"]) == 0
    assert json.loads(capsys.readouterr().out)["status"]["worker"]["running"] == 2
    t_end = time.time() + 10
    log = ""
    while time.time() < t_end and "rank 1 2" not in log:
        log = c.logs("demo-worker-1")
        time.sleep(0.1)
    assert "rank 1 2" in log
    assert pdoctl(["--server", url, "scale", "demo", "--replicas", "3"]) == 0
    t_end = time.time() + 20
    while time.time() < t_end and len(c.pods("demo")) != 3:
        time.sleep(0.1)
    assert len(c.pods("demo")) == 3
    assert pdoctl(["--server", url, "events", "demo"]) == 0
    assert "Created" in capsys.readouterr().out
    assert pdoctl(["--server", url, "delete", "demo"]) == 0
    t_end = time.time() + 20
    while time.time() < t_end and any(j["metadata"]["name"] == "demo" for j in c.list()):
        time.sleep(0.1)
    assert not any(j["metadata"]["name"] == "demo" for j in c.list())


def test_pdoctl_validate_rejects_bad_schema(tmp_path, capsys):
    bad = tmp_path / "bad.yaml"
    bad.write_text("apiVersion: batch.paddlepaddle.org/v1\nkind: PaddleJob\nmetadata: {name: b}\n"
                   "spec: {worker: {replicas: two}}\n")
    assert pdoctl(["validate", "-f", str(bad)]) == 1
    assert "validation error" in capsys.readouterr().err
    for f in sorted(os.listdir(os.path.join(REPO, "deploy", "examples"))):
        assert pdoctl(["validate", "-f", os.path.join(REPO, "deploy", "examples", f)]) == 0
