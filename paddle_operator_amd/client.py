"""PaddleJob REST client + ``pdoctl`` CLI.

Works against any Kubernetes-compatible API server: ``pdo-manager
--backend=local`` (its built-in API on ``--api-bind-address``) or a real
cluster's apiserver (``--server https://… --token …``).  The reference's
client demo (client/client.go:30-97) builds a clientset, creates a
PaddleJob from a struct and prints it; this is the same surface plus the
day-2 verbs a user needs (watch, scale, logs, events, wait).

    pdoctl --server http://127.0.0.1:8082 apply -f deploy/examples/resnet.yaml
    pdoctl get                      # NAME STATUS MODE AGE (the CRD printer columns)
    pdoctl scale resnet --role worker --replicas 4
    pdoctl wait resnet --phase Running --timeout 60
    pdoctl logs resnet-worker-0
    pdoctl delete resnet
"""
from __future__ import annotations

import argparse
import json
import os
import ssl
import sys
import time
import urllib.error
import urllib.parse
import urllib.request
from typing import Iterator, List, Optional

import yaml

from .api import types as T


class ApiError(RuntimeError):
    def __init__(self, code: int, body: str):
        super().__init__(f"HTTP {code}: {body[:300]}")
        self.code = code
        self.body = body


class PaddleJobClient:
    def __init__(self, server: str = "http://127.0.0.1:8082", token: str = "", insecure: bool = False,
                 namespace: str = "default", timeout: float = 10.0):
        self.server = server.rstrip("/")
        self.token = token
        self.ns = namespace
        self.timeout = timeout
        self.ctx = ssl._create_unverified_context() if insecure else None

    # ------------------------------------------------------------------ http
    def _req(self, method: str, path: str, body=None, ctype="application/json", stream=False):
        data = None
        if body is not None:
            data = body if isinstance(body, bytes) else json.dumps(body).encode()
        headers = {"Content-Type": ctype, "Accept": "application/json"}
        if self.token:
            headers["Authorization"] = f"Bearer {self.token}"
        req = urllib.request.Request(self.server + path, data=data, method=method, headers=headers)
        try:
            r = urllib.request.urlopen(req, timeout=None if stream else self.timeout, context=self.ctx)
        except urllib.error.HTTPError as e:
            raise ApiError(e.code, e.read().decode(errors="replace")) from None
        if stream:
            return r
        raw = r.read()
        r.close()
        if "json" in (r.headers.get("Content-Type") or "json"):
            return json.loads(raw or b"{}")
        return raw.decode(errors="replace")

    def _jobs(self, ns=None, name=""):
        p = f"/apis/{T.GROUP}/{T.VERSION}/namespaces/{ns or self.ns}/{T.PLURAL}"
        return p + (f"/{name}" if name else "")

    # ------------------------------------------------------------------ jobs
    def create(self, job: dict) -> dict:
        return self._req("POST", self._jobs(job.get("metadata", {}).get("namespace")), job)

    def get(self, name: str, ns=None) -> dict:
        return self._req("GET", self._jobs(ns, name))

    def list(self, ns=None) -> List[dict]:
        return self._req("GET", self._jobs(ns))["items"]

    def update(self, job: dict) -> dict:
        md = job["metadata"]
        return self._req("PUT", self._jobs(md.get("namespace"), md["name"]), job)

    def apply(self, job: dict) -> dict:
        md = job.setdefault("metadata", {})
        md.setdefault("namespace", self.ns)
        try:
            cur = self.get(md["name"], md["namespace"])
        except ApiError as e:
            if e.code != 404:
                raise
            return self.create(job)
        job = dict(job)
        job["metadata"] = dict(md, resourceVersion=cur["metadata"].get("resourceVersion"))
        return self.update(job)

    def delete(self, name: str, ns=None) -> dict:
        return self._req("DELETE", self._jobs(ns, name))

    def scale(self, name: str, role: str, replicas: int, ns=None, retries: int = 5) -> dict:
        for i in range(retries):
            job = self.get(name, ns)
            if role not in job["spec"]:
                raise ValueError(f"job {name} has no role {role!r}")
            job["spec"][role]["replicas"] = int(replicas)
            try:
                return self.update(job)
            except ApiError as e:
                if e.code != 409 or i == retries - 1:
                    raise
        raise RuntimeError("unreachable")

    def watch(self, ns=None) -> Iterator[dict]:
        r = self._req("GET", self._jobs(ns) + "?watch=true", stream=True)
        for line in r:
            line = line.strip()
            if line:
                yield json.loads(line)

    def wait(self, name: str, phase: str = "Running", timeout: float = 300.0, ns=None, poll: float = 0.2) -> dict:
        t_end = time.time() + timeout
        while True:
            job = self.get(name, ns)
            cur = (job.get("status") or {}).get("phase")
            if cur == phase:
                return job
            if cur in ("Failed", "Completed") and cur != phase:
                raise RuntimeError(f"{name} reached terminal phase {cur} while waiting for {phase}")
            if time.time() > t_end:
                raise TimeoutError(f"{name}: phase {cur!r} after {timeout}s (want {phase})")
            time.sleep(poll)

    # ------------------------------------------------------------------ pods / events
    def pods(self, job: str, ns=None) -> List[dict]:
        items = self._req("GET", f"/api/v1/namespaces/{ns or self.ns}/pods")["items"]
        out = []
        for p in items:
            for ref in p["metadata"].get("ownerReferences") or []:
                if ref.get("kind") == T.KIND and ref.get("name") == job:
                    out.append(p)
        return sorted(out, key=lambda p: p["metadata"]["name"])

    def logs(self, pod: str, ns=None, container: str = "", limit_bytes: int = 0) -> str:
        q = {}
        if container:
            q["container"] = container
        if limit_bytes:
            q["limitBytes"] = str(limit_bytes)
        qs = ("?" + urllib.parse.urlencode(q)) if q else ""
        return self._req("GET", f"/api/v1/namespaces/{ns or self.ns}/pods/{pod}/log{qs}")

    def events(self, involved: str = "", ns=None) -> List[dict]:
        items = self._req("GET", f"/api/v1/namespaces/{ns or self.ns}/events")["items"]
        if involved:
            items = [e for e in items if e.get("involvedObject", {}).get("name") == involved]
        return items


# ---------------------------------------------------------------------------- CLI
def _age(ts: Optional[str]) -> str:
    if not ts:
        return "<unknown>"
    try:
        t = time.mktime(time.strptime(ts, "%Y-%m-%dT%H:%M:%SZ")) - time.timezone
    except ValueError:
        return "<unknown>"
    s = max(0, int(time.time() - t))
    for unit, n in (("d", 86400), ("h", 3600), ("m", 60)):
        if s >= n:
            return f"{s // n}{unit}"
    return f"{s}s"


def _load_docs(path: str) -> List[dict]:
    text = sys.stdin.read() if path == "-" else open(path).read()
    if path.endswith(".json"):
        d = json.loads(text)
        return d if isinstance(d, list) else [d]
    return [d for d in yaml.safe_load_all(text) if d]


def _table(rows: List[List[str]]) -> str:
    w = [max(len(r[i]) for r in rows) for i in range(len(rows[0]))]
    return "\n".join("   ".join(c.ljust(w[i]) for i, c in enumerate(r)).rstrip() for r in rows)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="pdoctl", description="PaddleJob client (pdo)")
    ap.add_argument("--server", default=os.environ.get("PDO_SERVER", "http://127.0.0.1:8082"))
    ap.add_argument("--token", default=os.environ.get("PDO_TOKEN", ""))
    ap.add_argument("--insecure-skip-tls-verify", action="store_true")
    ap.add_argument("-n", "--namespace", default="default")
    sp = ap.add_subparsers(dest="cmd", required=True)
    p = sp.add_parser("apply")
    p.add_argument("-f", "--filename", required=True)
    p = sp.add_parser("create")
    p.add_argument("-f", "--filename", required=True)
    p = sp.add_parser("get")
    p.add_argument("name", nargs="?")
    p.add_argument("-o", "--output", choices=["wide", "json", "yaml"], default="")
    p = sp.add_parser("delete")
    p.add_argument("name")
    p = sp.add_parser("scale")
    p.add_argument("name")
    p.add_argument("--role", default="worker", choices=list(T.ROLE_ORDER))
    p.add_argument("--replicas", type=int, required=True)
    p = sp.add_parser("wait")
    p.add_argument("name")
    p.add_argument("--phase", default="Running")
    p.add_argument("--timeout", type=float, default=300)
    p = sp.add_parser("watch")
    p = sp.add_parser("pods")
    p.add_argument("name")
    p = sp.add_parser("logs")
    p.add_argument("pod")
    p.add_argument("-c", "--container", default="")
    p.add_argument("--limit-bytes", type=int, default=0)
    p = sp.add_parser("events")
    p.add_argument("name", nargs="?", default="")
    p = sp.add_parser("validate")
    p.add_argument("-f", "--filename", required=True)
    a = ap.parse_args(argv)
    c = PaddleJobClient(a.server, a.token, a.insecure_skip_tls_verify, a.namespace)
    try:
        if a.cmd in ("apply", "create"):
            for doc in _load_docs(a.filename):
                T.validate(doc)
                doc.setdefault("metadata", {}).setdefault("namespace", a.namespace)
                out = c.apply(doc) if a.cmd == "apply" else c.create(doc)
                print(f"paddlejob.{T.GROUP}/{out['metadata']['name']} {'configured' if a.cmd == 'apply' else 'created'}")
        elif a.cmd == "validate":
            for doc in _load_docs(a.filename):
                T.validate(doc)
                print(f"{doc['metadata']['name']}: valid")
        elif a.cmd == "get":
            jobs = [c.get(a.name)] if a.name else c.list()
            if a.output == "json":
                print(json.dumps(jobs if not a.name else jobs[0], indent=2))
            elif a.output == "yaml":
                print(yaml.safe_dump(jobs if not a.name else jobs[0], sort_keys=False))
            else:
                rows = [["NAME", "STATUS", "MODE", "AGE"] + (["PS", "WORKER", "HETER"] if a.output == "wide" else [])]
                for j in jobs:
                    st = j.get("status") or {}
                    r = [j["metadata"]["name"], st.get("phase", ""), st.get("mode", ""),
                         _age(j["metadata"].get("creationTimestamp"))]
                    if a.output == "wide":
                        for role in T.ROLE_ORDER:
                            rs = st.get(role) or {}
                            spec = (j["spec"].get(role) or {}).get("replicas")
                            r.append("" if spec is None else f"{rs.get('running', 0)}/{spec}")
                    rows.append(r)
                print(_table(rows))
        elif a.cmd == "delete":
            c.delete(a.name)
            print(f"paddlejob.{T.GROUP} \"{a.name}\" deleted")
        elif a.cmd == "scale":
            c.scale(a.name, a.role, a.replicas)
            print(f"paddlejob.{T.GROUP}/{a.name} scaled ({a.role}={a.replicas})")
        elif a.cmd == "wait":
            c.wait(a.name, a.phase, a.timeout)
            print(f"paddlejob.{T.GROUP}/{a.name} condition met ({a.phase})")
        elif a.cmd == "watch":
            for ev in c.watch():
                st = ev["object"].get("status") or {}
                print(f"{ev['type']:8s} {ev['object']['metadata']['name']} {st.get('phase', '')} {st.get('mode', '')}",
                      flush=True)
        elif a.cmd == "pods":
            rows = [["NAME", "PHASE", "IP", "NODE"]]
            for p in c.pods(a.name):
                st = p.get("status") or {}
                rows.append([p["metadata"]["name"], st.get("phase", ""), st.get("podIP", ""),
                             p["spec"].get("nodeName", "")])
            print(_table(rows))
        elif a.cmd == "logs":
            sys.stdout.write(c.logs(a.pod, container=a.container, limit_bytes=a.limit_bytes))
        elif a.cmd == "events":
            rows = [["TYPE", "REASON", "OBJECT", "MESSAGE"]]
            for e in c.events(a.name):
                rows.append([e.get("type", ""), e.get("reason", ""), e["involvedObject"].get("name", ""),
                             e.get("message", "")])
            print(_table(rows))
    except ApiError as e:
        print(f"Error from server: {e}", file=sys.stderr)
        return 1
    except (TimeoutError, RuntimeError, ValueError) as e:
        print(f"error: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
