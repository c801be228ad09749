"""Elastic agent: KV membership → rendezvous → supervised RCCL worker.

The reference operator only keeps ``/paddle/<ns>-<name>/np`` in etcd in sync
with ``spec.worker.replicas`` (controllers/paddlejob_elastic.go:27-55) and
gives elastic pods OnFailure restarts plus the PADDLE_ELASTIC_* env
(controllers/paddlejob_helper.go:333-348); re-rendezvous is left to the Paddle
image.  An RCCL communicator cannot be resized, so pdo's agent owns the
worker process and rebuilds the world on every membership/np change:

KV layout under ``/paddle/<job-id>/`` (pdo-kv, etcd-v3 JSON gateway):

* ``np``                — desired world size; the agent creates it from
  PADDLE_ELASTIC_NP if absent (the controller never creates it, only updates).
* ``nodes/<id>``        — membership, value ``{"id","host","port","lease","inc"}``,
  bound to a lease of ``ttl`` seconds kept alive by the agent: a killed pod
  drops out after ``ttl`` without anyone deleting it.
* ``rdzv/<gen>/<id>``   — per-generation arrival barrier.  ``gen`` is a digest
  of (np, the first np members' (id, lease, inc)), so every agent that sees
  the same membership computes the same generation, the same rank order and
  the same TCPStore port (``PADDLE_PORT + 2 + gen % 16`` on rank 0's host;
  each pod owns 20 ports, paddlejob_helper.go:215-279).  A pod that was killed
  and restarted in place (OnFailure, paddlejob_helper.go:366-374) comes back
  with a new lease, and an agent whose worker crashed bumps ``inc``: either
  way the generation id changes, so no stale arrival key or still-bound
  TCPStore port of the previous generation can be mistaken for the new one.
* ``done/<id>``         — written when a worker finished all steps.

Loop: register → wait for ≥ np live members (``PADDLE_ELASTIC_TIMEOUT``) →
barrier on ``rdzv/<gen>`` → spawn ``pdo-launch --worker`` with RANK/WORLD_SIZE/
MASTER_* → watch np + membership every ``poll`` s; on change SIGTERM the
worker (rank 0 checkpoints in its SIGTERM handler) and rendezvous again; on
worker failure, wait up to one lease TTL for the membership to change (a
dead peer is the usual cause: its lease expires), otherwise count a restart
(``max_restarts``) and bump ``inc`` so every peer re-forms the world.
Workers resume from the newest checkpoint, whose flat-arena layout does not
depend on the world size.

xGMI layout (``--nproc-per-pod N``): a member is a pod holding N GPUs (one
pod per node, ``amd.com/gpu: 8``), so RCCL connects its local ranks peer to
peer over xGMI instead of through sockets between one-GPU pods.  ``np`` stays
the pod count (the controller's ``worker.replicas``); each generation is a
world of np·N ranks, pod rank p's local rank i being global rank p·N + i.  The
agent never touches HIP: it forks its N workers fresh for every generation
(new processes, so every RCCL communicator and HIP context is new), and the
first local rank to fail takes its siblings down — a failure of the pod, as
one worker's failure was with N = 1.
"""
from __future__ import annotations

import hashlib
import json
import os
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Tuple

from ..kv.client import KVClient, KVError

STORE_BASE_OFFSET = 2
STORE_PORTS = 16


def _log(msg):
    print(f"[pdo-elastic {time.strftime('%H:%M:%S')}] {msg}", flush=True)


class ElasticAgent:
    def __init__(self, kv: KVClient, job_id: str, member_id: int, host: str, port: int, np_default: int,
                 timeout: float = 60.0, ttl: int = 6, poll: float = 0.25, max_restarts: int = 3, nproc: int = 1):
        self.kv = kv
        self.nproc = max(1, int(nproc))
        self.job = job_id
        self.id = int(member_id)
        self.host, self.port = host, int(port)
        self.np_default = int(np_default)
        self.timeout = timeout
        self.ttl = ttl
        self.poll = poll
        self.max_restarts = max_restarts
        self.prefix = f"/paddle/{job_id}/"
        self.lease = 0
        self.inc = 0
        self._ka = None
        self._lease_lost = threading.Event()
        self.reregistrations = 0
        self.procs: List[subprocess.Popen] = []
        self.history: List[dict] = []

    # ------------------------------------------------------------ membership
    def register(self):
        self.kv.put_if_absent(self.prefix + "np", str(self.np_default))
        self._grant()

    def _grant(self):
        self._lease_lost.clear()
        self.lease = self.kv.lease_grant(self.ttl)
        self._announce()
        self._ka = self.kv.keepalive_thread(self.lease, self.ttl, on_lost=self._lease_lost.set)

    def ensure_registered(self) -> bool:
        """Re-join after the membership lease was lost (the KV was unreachable
        for more than a TTL): a new lease and a fresh ``nodes/`` record.  The
        new lease id changes the generation plan, so peers re-form the world
        with this member instead of it timing out in rendezvous.  True if a
        re-registration happened."""
        if not self._lease_lost.is_set():
            return False
        try:
            if self._ka is not None:
                self._ka.set()
            self._grant()
        except KVError as e:  # KV still away: the next poll retries
            _log(f"re-register failed ({e}); retrying")
            self._lease_lost.set()
            return False
        self.reregistrations += 1
        _log(f"membership lease lost → re-registered with lease {self.lease}")
        return True

    def _announce(self):
        self.kv.put(self.prefix + f"nodes/{self.id:06d}",
                    json.dumps({"id": self.id, "host": self.host, "port": self.port, "lease": self.lease,
                                "inc": self.inc}), lease=self.lease)

    def bump(self):
        """This member's worker failed on its own: force a fresh generation."""
        self.inc += 1
        self._announce()

    def deregister(self):
        if self._ka is not None:
            self._ka.set()
        try:
            if self.lease:
                self.kv.lease_revoke(self.lease)
        except Exception:
            pass

    def np(self) -> int:
        v = self.kv.get(self.prefix + "np")
        try:
            return int(v) if v is not None else self.np_default
        except ValueError:
            return self.np_default

    def members(self) -> List[dict]:
        kvs = self.kv.get_prefix(self.prefix + "nodes/")
        out = [json.loads(v) for _, v in sorted(kvs.items())]
        return sorted(out, key=lambda m: m["id"])

    @staticmethod
    def plan(np_: int, members: List[dict]) -> Tuple[int, List[dict]]:
        """Deterministic generation id + rank order for (np, membership)."""
        chosen = members[:np_]
        ident = [[m["id"], m.get("lease", 0), m.get("inc", 0)] for m in chosen]
        h = hashlib.sha1(json.dumps([np_, ident]).encode()).hexdigest()
        return int(h[:8], 16), chosen

    # ------------------------------------------------------------ rendezvous
    def rendezvous(self) -> Optional[dict]:
        """Block until a generation forms that includes this member.

        Returns the world description, or None on timeout."""
        deadline = time.time() + self.timeout
        while time.time() < deadline:
            self.ensure_registered()
            np_ = self.np()
            mem = self.members()
            if len(mem) < np_:
                time.sleep(self.poll)
                continue
            gen, chosen = self.plan(np_, mem)
            ids = [m["id"] for m in chosen]
            if self.id not in ids:  # surplus member: stand by until np grows / someone leaves
                time.sleep(self.poll)
                deadline = time.time() + self.timeout
                continue
            key = self.prefix + f"rdzv/{gen:08x}/"
            self.kv.put(key + f"{self.id:06d}", "1", lease=self.lease)
            # every chosen member must arrive while the plan stays valid
            t_bar = time.time() + min(10.0, max(1.0, deadline - time.time()))
            while time.time() < t_bar:
                if len(self.kv.get_prefix(key)) >= np_:
                    master = chosen[0]
                    return {"gen": gen, "np": np_, "rank": ids.index(self.id), "ids": ids,
                            "master_addr": master["host"],
                            "master_port": master["port"] + STORE_BASE_OFFSET + gen % STORE_PORTS}
                if self.plan(self.np(), self.members())[0] != gen:
                    break
                time.sleep(self.poll / 2)
        return None

    def gen_done(self, world: dict) -> bool:
        """A peer of this generation already finished all steps: the job is
        complete, and peers leaving now is teardown, not a scale event."""
        for v in self.kv.get_prefix(self.prefix + "done/").values():
            try:
                if json.loads(v).get("gen") == world["gen"]:
                    return True
            except (ValueError, AttributeError):
                continue
        return False

    def changed(self, world: dict) -> bool:
        np_ = self.np()
        mem = self.members()
        return len(mem) < np_ or self.plan(np_, mem)[0] != world["gen"]

    # ------------------------------------------------------------ supervision
    def spawn(self, world: dict, worker_argv: List[str]) -> List[subprocess.Popen]:
        """This pod's nproc local ranks of generation ``world``."""
        n = self.nproc
        procs = []
        for i in range(n):
            env = dict(os.environ)
            env.update({"RANK": str(world["rank"] * n + i), "WORLD_SIZE": str(world["np"] * n),
                        "LOCAL_RANK": str(i), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": world["master_addr"],
                        "MASTER_PORT": str(world["master_port"]), "PDO_ELASTIC_GEN": f"{world['gen']:08x}"})
            cmd = [sys.executable, "-m", "paddle_operator_amd.launch", "--worker"] + worker_argv
            # own session so stop_workers() can signal the worker's whole group; but
            # a pod kill (SIGKILL to the agent's group, as a container runtime
            # would kill the container) must take the worker down too
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True, preexec_fn=_die_with_parent))
        return procs

    def poll_workers(self) -> Optional[int]:
        """None while any local rank runs and none failed; else the pod's exit
        status — 0 once every local rank finished, or the first failure's."""
        rcs = [p.poll() for p in self.procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            return bad[0]
        return 0 if all(rc == 0 for rc in rcs) else None

    def wait_workers(self, timeout: float) -> int:
        """Wait for the local ranks to finish: the first non-zero exit stops the
        others and is returned; past ``timeout`` every rank is stopped (rc 124)."""
        t_end = time.time() + timeout
        while True:
            rc = self.poll_workers()
            if rc is not None:
                if rc != 0:
                    self.stop_workers(5.0)
                return rc
            if time.time() >= t_end:
                _log(f"workers still running {timeout:.0f}s after the generation completed: stopping them")
                self.stop_workers(5.0)
                return 124
            time.sleep(self.poll / 2)

    def stop_workers(self, grace: float = 20.0):
        live = [p for p in self.procs if p.poll() is None]
        for p in live:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        t_end = time.time() + grace
        for p in live:
            try:
                p.wait(max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def run(self, worker_argv: List[str]) -> int:
        self.register()
        restarts = 0
        try:
            while True:
                t0 = time.time()
                world = self.rendezvous()
                if world is None:
                    _log(f"rendezvous timed out after {self.timeout}s")
                    return 3
                _log(f"gen {world['gen']:08x}: pod rank {world['rank']}/{world['np']} × {self.nproc} local "
                     f"master {world['master_addr']}:{world['master_port']} (rdzv {time.time() - t0:.2f}s)")
                self.history.append(world)
                self.procs = self.spawn(world, worker_argv)
                while True:
                    rc = self.poll_workers()
                    if rc is not None:
                        break
                    self.ensure_registered()
                    if self.changed(world):
                        if self.gen_done(world):
                            # generation completed: let this pod's workers finish too —
                            # polled with a deadline: a local rank that fails now must
                            # not leave its siblings hanging in a collective
                            rc = self.wait_workers(self.timeout)
                            break
                        _log("membership/np changed → stopping workers for re-rendezvous")
                        self.stop_workers()
                        rc = None
                        break
                    time.sleep(self.poll)
                if rc is None:
                    continue
                if rc == 0:
                    self.kv.put(self.prefix + f"done/{self.id:06d}", json.dumps({"gen": world["gen"]}))
                    return 0
                self.stop_workers(5.0)  # a failed local rank takes its siblings down
                # a dead peer usually takes this worker down with it before
                # its lease has expired: give the membership one TTL to move
                t_end = time.time() + self.ttl + 2 * self.poll
                while not self.changed(world) and time.time() < t_end:
                    time.sleep(self.poll)
                if self.changed(world):
                    _log(f"worker exited rc={rc} after a membership change → re-rendezvous")
                    continue  # a peer left: not this worker's fault
                restarts += 1
                _log(f"worker exited rc={rc}; restart {restarts}/{self.max_restarts}")
                if restarts > self.max_restarts:
                    return rc
                self.bump()
        finally:
            self.stop_workers(5.0)
            self.deregister()


def _die_with_parent():
    """Child side of spawn(): SIGKILL this worker when the agent dies."""
    try:
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except OSError:
        pass


def _strip(argv: List[str]) -> List[str]:
    """Worker argv: the agent's own flags removed (each worker is one rank)."""
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in ("--elastic", "--worker"):
            continue
        if a == "--nproc-per-pod":
            skip = True
            continue
        if a.startswith("--nproc-per-pod="):
            continue
        out.append(a)
    return out


def run_agent(args, jenv, argv: List[str]) -> int:
    eps = jenv.kv_endpoints()
    if not eps:
        raise SystemExit("elastic mode needs PADDLE_ELASTIC_SERVER (or PDO_KV)")
    agent = ElasticAgent(KVClient(eps), jenv.elastic_job_id or jenv.job_key(), jenv.trainer_id, jenv.pod_ip,
                         jenv.port, jenv.elastic_np or jenv.trainers_num, timeout=float(jenv.elastic_timeout),
                         ttl=int(os.environ.get("PDO_ELASTIC_TTL", "6")), nproc=getattr(args, "nproc_per_pod", 1))
    signal.signal(signal.SIGTERM, lambda *a: sys.exit(143))
    return agent.run(_strip(argv))
