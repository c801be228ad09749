"""Python driver of the native control plane (``_pdo_core``).

``LocalCluster`` is the local backend (object store + gang scheduler +
kubelet-lite agents + PaddleJob controller + pdo-kv) as one object that tests
and the launch benchmark drive directly; ``pdo-manager --backend=local``
runs the same C++ code as a daemon with a Kubernetes-compatible REST API.

Reference behaviour parity (controllers/paddlejob_controller.go) is in the
native planner; ``mode="compat"`` reproduces the reference's sequencing.
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

from .. import _native
from ..api import types as T


def core():
    return _native.require_core()


class LocalCluster:
    """Local backend.

    Options (all keyword): mode ("fast"|"compat"), agent ("sim"|"exec"),
    nodes ([{name, gpus, ip, gpu_cpulists}]), init_image, volcano, elastic_kv,
    workers, virtual_clock, sandbox_root, sim_ip_delay, sim_start_delay,
    sim_run_s, kubelet_config_retry_s, port_range, namespace.
    """

    def __init__(self, **opts):
        if opts.pop("zygote", False):
            # per-node warm launcher: pods whose entry point is bin/pdo-launch fork
            # from a pre-imported interpreter (launch/zygote.py)
            import os
            import sys
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            pp = os.environ.get("PYTHONPATH", "")
            if root not in pp.split(os.pathsep):
                os.environ["PYTHONPATH"] = root + (os.pathsep + pp if pp else "")
            opts["zygote_cmd"] = [sys.executable, "-m", "paddle_operator_amd.launch.zygote"]
        if opts.get("agent") == "exec" and "ip_block_base" not in opts:
            # every pod has its own 127.<block>.x.y; a per-process block keeps
            # clusters of concurrently running processes (xdist) off each other's
            # :2379 rendezvous ports
            import os
            opts["ip_block_base"] = 2 + os.getpid() % 200
        self._c = core().Cluster(**opts)
        self.opts = opts
        self.url: Optional[str] = None

    # -- objects -------------------------------------------------------------
    def apply(self, obj: dict, kind: Optional[str] = None) -> dict:
        return self._c.apply(kind or obj["kind"], obj)

    def create(self, obj: dict, kind: Optional[str] = None) -> dict:
        return self._c.create(kind or obj["kind"], obj)

    def get(self, kind: str, name: str, ns: str = "default") -> Optional[dict]:
        return self._c.get(kind, ns, name)

    def job(self, name: str, ns: str = "default") -> Optional[dict]:
        return self._c.get(T.KIND, ns, name)

    def list(self, kind: str, ns: str = "", labels: Optional[dict] = None, owner: str = "") -> List[dict]:
        return self._c.list(kind, ns, labels or {}, owner)

    def pods(self, job: str, ns: str = "default") -> List[dict]:
        return self._c.list("Pod", ns, {}, job)

    def events(self, ns: str = "default", involved: Optional[str] = None) -> List[dict]:
        evs = self._c.list("Event", ns, {}, "")
        if involved:
            evs = [e for e in evs if e["involvedObject"]["name"] == involved]
        return evs

    def update(self, obj: dict, kind: Optional[str] = None) -> dict:
        return self._c.update(kind or obj["kind"], obj)

    def update_status(self, obj: dict, kind: Optional[str] = None) -> dict:
        return self._c.update_status(kind or obj["kind"], obj)

    def delete(self, kind: str, name: str, ns: str = "default") -> bool:
        return self._c.delete(kind, ns, name)

    def scale(self, name: str, role: str, replicas: int, ns: str = "default") -> dict:
        j = self.job(name, ns)
        j["spec"][role]["replicas"] = replicas
        return self._c.update(T.KIND, j)

    # -- driving -------------------------------------------------------------
    def tick(self) -> bool:
        return self._c.tick()

    def settle(self, max_s: float = 5.0) -> int:
        return self._c.settle(max_s)

    def run_for(self, seconds: float, step: float = 0.01) -> int:
        return self._c.run_for(seconds, step)

    def now(self) -> float:
        return self._c.now()

    def advance(self, dt: float):
        self._c.advance(dt)

    def wait(self, pred: Callable[[], bool], timeout: float = 10.0, step: float = 0.01) -> bool:
        """Tick until ``pred()`` holds; virtual time if the cluster has a virtual clock."""
        virtual = bool(self.opts.get("virtual_clock"))
        t_end = (self.now() if virtual else time.time()) + timeout
        while True:
            if pred():
                return True
            now = self.now() if virtual else time.time()
            if now >= t_end:
                return pred()
            self._c.run_for(step, step if virtual else min(step, 0.005))

    def wait_phase(self, name: str, phase: str, ns: str = "default", timeout: float = 10.0) -> bool:
        return self.wait(lambda: ((self.job(name, ns) or {}).get("status") or {}).get("phase") == phase,
                         timeout)

    # -- pods / faults -----------------------------------------------------------
    def exec(self, pod: str, container: str, argv: List[str], ns: str = "default") -> bool:
        return self._c.exec(ns, pod, container, list(argv))

    def kill(self, pod: str, sig: int = 9, ns: str = "default") -> bool:
        return self._c.kill(ns, pod, sig)

    def sim_exit(self, pod: str, code: int = 0, ns: str = "default") -> bool:
        return self._c.sim_exit(ns, pod, code)

    def sandbox(self, pod: str, ns: str = "default") -> str:
        return self._c.sandbox(ns, pod)

    def set_pod_status(self, pod: str, ns: str = "default", **status) -> dict:
        """Test hook: overwrite fields of a pod's status (fake kubelet)."""
        p = self._c.get("Pod", ns, pod)
        p.setdefault("status", {}).update(status)
        p["metadata"].pop("resourceVersion", None)
        return self._c.update_status("Pod", p)

    # -- kv --------------------------------------------------------------------
    def kv_put(self, key: str, value: str):
        return self._c.kv_put(key, value)

    def kv_get(self, key: str) -> Optional[str]:
        return self._c.kv_get(key)

    def kv_delete(self, key: str):
        return self._c.kv_delete(key)

    # -- misc --------------------------------------------------------------------
    def free_gpus(self) -> Dict[str, int]:
        return self._c.free_gpus()

    def reconcile(self, name: str, ns: str = "default"):
        return self._c.reconcile(ns, name)

    def serve(self, addr: str = "127.0.0.1:0") -> str:
        port = self._c.serve(addr)
        host = addr.rsplit(":", 1)[0] or "127.0.0.1"
        self.url = f"http://{host}:{port}"
        return self.url

    def start(self):
        self._c.start()

    def zygotes_ready(self) -> bool:
        return self._c.zygotes_ready()

    def zygote_status(self) -> Dict[str, Optional[dict]]:
        """Per node: the warm launcher's slot table (launch/zygote.py ``status``)."""
        import glob
        import os

        from ..launch.zygote import query_status
        root = self.opts.get("sandbox_root") or ""
        return {os.path.basename(os.path.dirname(p)): query_status(p)
                for p in sorted(glob.glob(os.path.join(root, "*", "zygote.sock")))}

    def wait_warm(self, timeout: float = 120.0) -> bool:
        """Block until every node's GPU-warm slots are up (node idle)."""
        deadline = time.time() + timeout
        while time.time() < deadline:
            st = self.zygote_status()
            if st and all(z is not None and all(s["ready"] and s.get("n_ready", 1) >= s.get("n", 1)
                                                for s in z["slots"].values())
                          and (len(z["slots"]) + len(z.get("failed") or {})) >= len(z["devices"])
                          for z in st.values()):
                return True
            time.sleep(0.02)
        return False

    def stop(self):
        self._c.stop()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def metrics() -> str:
    return core().metrics()


def metric(name: str, **labels) -> float:
    return core().metric(name, labels)
