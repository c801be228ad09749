"""Rank bootstrap on MI355X: device affinity → RCCL communicator → readiness.

Order matters on ROCm (BASELINE north star: "RCCL-init / HIP device-affinity
path"):

1. ``pin``: CPU affinity to the GPU's NUMA-local cores (sysfs, no HIP).
2. ``hipSetDevice(local_rank)`` (``torch.cuda.set_device``) BEFORE any other
   HIP call, so the RCCL communicator and every allocation bind the right GPU.
3. ``init_process_group("nccl")`` — on ROCm the nccl backend IS RCCL; the
   unique id travels through rank 0's TCPStore (or pdo-kv for elastic jobs);
   ``device_id`` makes the communicator eager (created now, not lazily at the
   first collective), so "ready" really means the xGMI rings are up.
4. Optional intra-node IPC probe: every rank exports a staging buffer with
   ``hipIpcGetMemHandle``; peers on the same node open it
   (``hipIpcOpenMemHandle``) and copy over xGMI — validates peer access and
   measures per-pair bandwidth before training (bucket sizing input).
5. Warm-up all-reduce, then a readiness record in pdo-kv
   (``/pdo/<job>/ready/<rank>``) and a ``PDO_READY`` log line.
"""
from __future__ import annotations

import datetime
import json
import os
import socket
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .. import _native
from ..utils import topology


@dataclass
class Bootstrapped:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str
    t_start: float
    t_pg: float = 0.0
    t_ready: float = 0.0
    ipc_gbps: Optional[dict] = None
    # wall-clock split of bootstrap (s): entry = process start → init() call
    # (interpreter + imports), hip = device init, comm = communicator init,
    # warm = warm-up all-reduce
    phases: Optional[dict] = None


def _wait_port(host: str, port: int, timeout_s: float, poll: float = 0.002) -> bool:
    deadline = time.time() + timeout_s
    while time.time() < deadline:
        try:
            with socket.create_connection((host, port), timeout=0.5):
                return True
        except OSError:
            time.sleep(poll)
    return False


_STORE = []  # keeps rank 0's store (it owns the listening socket) alive for the job


def _bound_store(host: str, port: int, world: int, timeout_s: int):
    """Rank 0's c10d TCPStore listening on ``host`` only.

    c10d binds its store to the wildcard address.  On Kubernetes every pod has
    its own network namespace, but the local backend's exec agent runs pods as
    processes with one loopback IP each, so two concurrent jobs' rank 0 both
    wanting ``PADDLE_PORT + 1`` collided (EADDRINUSE).  A socket bound to the
    pod's own address and handed over as ``master_listen_fd`` keeps them apart.
    Returns None when ``host`` is not a local address (a service name or
    ClusterIP): then c10d's default wildcard store is used."""
    try:
        ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        ls.bind((socket.gethostbyname(host), port))
        ls.listen(1024)
    except OSError:
        return None
    # the descriptor's ownership moves to c10d's server: detached, the Python
    # socket object can never close it a second time (a number the process
    # may meanwhile have reused for something else)
    fd = ls.detach()
    try:
        store = dist.TCPStore(host, port, world, True, datetime.timedelta(seconds=timeout_s),
                              wait_for_workers=False, master_listen_fd=fd)
    except BaseException:
        os.close(fd)
        raise
    _STORE.append(store)
    return store


def _env_int(k, d):
    return int(os.environ.get(k, str(d)))


def init(t_start: float, backend: Optional[str] = None, timeout_s: int = 300, ipc_probe: bool = False,
         store=None) -> Bootstrapped:
    t_entry = time.time()
    rank = _env_int("RANK", 0)
    world = _env_int("WORLD_SIZE", 1)
    local = _env_int("LOCAL_RANK", 0)
    # PDO_GPU_IDS (agent with PDO_GPU_VISIBILITY=all): every GPU is visible and
    # this pod's own ids are listed; else HIP_VISIBLE_DEVICES isolation → index
    ids = [int(x) for x in os.environ.get("PDO_GPU_IDS", "").split(",") if x.strip().isdigit()]
    index = ids[local] if local < len(ids) else local
    topology.pin_to_gpu(index)  # before HIP init: uses sysfs only
    gpu = torch.cuda.is_available()
    if backend is None:
        backend = "nccl" if gpu else "gloo"
    if gpu:
        torch.cuda.set_device(index)  # hipSetDevice
        torch.cuda.init()
        dev = torch.device("cuda", index)
    else:
        dev = torch.device("cpu")
    t_dev = time.time()
    b = Bootstrapped(rank, world, local, dev, backend, t_start)
    t_comm = t_dev
    # RCCL is brought up even for a 1-rank job: "ready" then always includes
    # communicator init, and the DDP code path is the one that runs at scale.
    # A CPU (gloo) world of 1 has nothing to rendezvous with.
    if (world > 1 or backend == "nccl") and not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        if store is not None:
            kw["store"] = store
        elif world == 1:
            kw["store"] = dist.HashStore()
        else:
            host, port = os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"])
            # explicit stores on every rank (an init_method URL would put the
            # process group's keys under a "default_pg" prefix on one side only)
            to = datetime.timedelta(seconds=timeout_s)
            if rank == 0:
                kw["store"] = (_bound_store(host, port, world, timeout_s)
                               or dist.TCPStore(host, port, world, True, to, wait_for_workers=False))
            else:
                # c10d's client connect retries back off to ~1 s; ranks forked
                # in the same ms as rank 0 would otherwise sleep through its bind
                _wait_port(host, port, timeout_s)
                kw["store"] = dist.TCPStore(host, port, world, False, to)
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
        t_comm = time.time()
        if ipc_probe and gpu:
            b.ipc_gbps = ipc_probe_run(dev)
        # warm-up: forces the communicator + first ring setup before "ready"
        t = torch.ones(1, device=dev)
        dist.all_reduce(t)
        if gpu:
            torch.cuda.synchronize(dev)
    b.t_pg = time.time()
    b.phases = {"entry": round(t_entry - t_start, 4), "hip": round(t_dev - t_entry, 4),
                "comm": round(t_comm - t_dev, 4), "warm": round(b.t_pg - t_comm, 4)}
    # entry split (zygote launches): client → zygote, parked behind a warming
    # slot, and handoff/fork → bootstrap.init inside the rank
    t_recv, t_disp = os.environ.get("PDO_T_ZYG_RECV"), os.environ.get("PDO_T_DISPATCH")
    if t_recv and t_disp:
        b.phases.update({"to_zygote": round(float(t_recv) - t_start, 4),
                         "park": round(float(t_disp) - float(t_recv), 4),
                         "rank_entry": round(t_entry - float(t_disp), 4)})
    return b


def ipc_probe_run(dev: torch.device, nbytes: int = 64 << 20) -> dict:
    """Exchange hipIpc handles with same-node peers and time a 64 MiB copy per pair."""
    m = _native.require_hip()
    rank, world = dist.get_rank(), dist.get_world_size()
    node = os.environ.get("PDO_NODE_NAME") or socket.gethostname()
    buf = torch.full((nbytes,), rank % 251, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    handle, off = m.ipc_get_handle(buf)
    rec = {"node": node, "pid": os.getpid(), "handle": handle.hex(), "offset": off,
           "device": torch.cuda.current_device(), "bdf": m.device_info(torch.cuda.current_device())["pci_bus_id"]}
    allrec = [None] * world
    dist.all_gather_object(allrec, rec)
    out = {}
    peers = [r for r, x in enumerate(allrec) if x["node"] == node and r != rank]
    local_dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    for r in peers:
        try:
            peer = m.ipc_open_handle(bytes.fromhex(allrec[r]["handle"]), nbytes, dev.index, allrec[r]["offset"])
        except RuntimeError as e:  # no peer access between the two GPUs
            out[r] = f"unavailable: {e}"
            continue
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(4):
            local_dst.copy_(peer, non_blocking=True)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / 4
        ok = bool((local_dst[:4096] == (r % 251)).all().item())
        out[r] = round(nbytes / dt / 1e9, 1) if ok else "mismatch"
        del peer
    dist.barrier()  # keep every exported buffer alive until all peers are done
    del buf
    return out


def report_ready(b: Bootstrapped, job_key: str, kv_endpoints: str = "", extra: Optional[dict] = None):
    b.t_ready = time.time()
    rec = {"rank": b.rank, "world": b.world, "local_rank": b.local_rank, "t_start": b.t_start, "t_pg": b.t_pg, "t_ready": b.t_ready,
           "host": socket.gethostname(), "pid": os.getpid(), "backend": b.backend}
    if os.environ.get("PDO_ELASTIC_GEN"):
        rec["gen"] = os.environ["PDO_ELASTIC_GEN"]
    if b.ipc_gbps is not None:
        rec["ipc_gbps"] = b.ipc_gbps
    if b.phases:
        rec["phases"] = b.phases
    # served by a GPU-warm slot of the node's zygote (HIP + RCCL code already loaded)
    rec["warm_slot"] = os.environ.get("PDO_WARM_SLOT_USED") == "1"
    if extra:
        rec.update(extra)
    line = "PDO_READY " + json.dumps(rec)
    print(line, flush=True)
    if kv_endpoints:
        from ..kv.client import KVClient
        try:
            KVClient(kv_endpoints).put(f"/pdo/{job_key}/ready/{b.rank}", json.dumps(rec))
        except Exception as e:  # readiness reporting must never kill a rank
            print(f"[pdo-launch] ready report to kv failed: {e}", flush=True)
    return rec
