"""GPU topology and device affinity for MI355X nodes (no HIP initialisation).

* ``gpu_topology()`` reads the link matrix from rocm_smi (``librocm_smi64``
  via ctypes: rsmi_topo_get_link_type / _link_weight / _numa_node_number /
  rsmi_dev_pci_id_get), falling back to the KFD sysfs topology.  On an
  8×MI355X node every GPU pair is one xGMI hop (fully connected, 7 links per
  GPU) — ring collectives are then bounded by one link per ring step, and
  RCCL runs up to 7 rings concurrently.
* ``numa_cpus(bdf)`` — the NUMA-local CPU set of a GPU (sysfs local_cpulist)
  used to pin each rank (``pin_to_gpu``).
* ``bucket_bytes_for(...)`` — all-reduce bucket size policy for xGMI (see
  parallel/ddp.py): large enough for a ring step per link to be
  bandwidth-bound, small enough to start overlapping early.
* ``gpu_count()`` — usable GPUs from KFD sysfs (no HIP init).

Nothing here touches the GPU runtime, so the manager / agent can call it
without initialising HIP (forking after HIP init is unsafe).
"""
from __future__ import annotations

import ctypes
import glob
import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

LINK_TYPES = {0: "undefined", 1: "pcie", 2: "xgmi", 3: "num"}


@dataclass
class GPU:
    index: int
    bdf: str = ""
    numa_node: int = -1
    cpus: List[int] = field(default_factory=list)


@dataclass
class Topology:
    gpus: List[GPU]
    link_type: List[List[str]]
    hops: List[List[int]]
    weight: List[List[int]]
    source: str

    @property
    def n(self):
        return len(self.gpus)

    def fully_connected_xgmi(self) -> bool:
        n = self.n
        return n > 1 and all(self.link_type[i][j] == "xgmi" and self.hops[i][j] == 1
                             for i in range(n) for j in range(n) if i != j)

    def to_dict(self):
        return {"gpus": [g.__dict__ for g in self.gpus], "link_type": self.link_type, "hops": self.hops,
                "weight": self.weight, "source": self.source,
                "fully_connected_xgmi": self.fully_connected_xgmi()}


def _parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for tok in s.strip().split(","):
        if not tok:
            continue
        if "-" in tok:
            a, b = tok.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(tok))
    return out


def numa_cpus(bdf: str) -> List[int]:
    for cand in (f"/sys/bus/pci/devices/{bdf}/local_cpulist", f"/sys/bus/pci/devices/{bdf.lower()}/local_cpulist"):
        try:
            with open(cand) as f:
                return _parse_cpulist(f.read())
        except OSError:
            pass
    return []


def _rsmi():
    for name in ("librocm_smi64.so.1", "librocm_smi64.so", "/opt/rocm/lib/librocm_smi64.so"):
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    return None


def _from_rsmi() -> Optional[Topology]:
    lib = _rsmi()
    if lib is None or lib.rsmi_init(ctypes.c_uint64(0)) != 0:
        return None
    try:
        n = ctypes.c_uint32(0)
        if lib.rsmi_num_monitor_devices(ctypes.byref(n)) != 0 or n.value == 0:
            return None
        gpus = []
        for i in range(n.value):
            bdfid = ctypes.c_uint64(0)
            bdf = ""
            if lib.rsmi_dev_pci_id_get(ctypes.c_uint32(i), ctypes.byref(bdfid)) == 0:
                v = bdfid.value
                # rsmi BDFID: domain<<32 | bus<<8 | device<<3 | function
                bdf = "%04x:%02x:%02x.%x" % ((v >> 32) & 0xffff, (v >> 8) & 0xff, (v >> 3) & 0x1f, v & 0x7)
            numa = ctypes.c_uint32(0)
            nn = numa.value if lib.rsmi_topo_get_numa_node_number(ctypes.c_uint32(i), ctypes.byref(numa)) == 0 \
                else -1
            gpus.append(GPU(i, bdf, nn if nn != 0xffffffff else -1, numa_cpus(bdf) if bdf else []))
        N = n.value
        lt = [["self"] * N for _ in range(N)]
        hops = [[0] * N for _ in range(N)]
        wt = [[0] * N for _ in range(N)]
        for a in range(N):
            for b in range(N):
                if a == b:
                    continue
                h = ctypes.c_uint64(0)
                t = ctypes.c_int(0)
                if lib.rsmi_topo_get_link_type(ctypes.c_uint32(a), ctypes.c_uint32(b), ctypes.byref(h),
                                               ctypes.byref(t)) == 0:
                    lt[a][b] = LINK_TYPES.get(t.value, str(t.value))
                    hops[a][b] = int(h.value)
                w = ctypes.c_uint64(0)
                if lib.rsmi_topo_get_link_weight(ctypes.c_uint32(a), ctypes.c_uint32(b), ctypes.byref(w)) == 0:
                    wt[a][b] = int(w.value)
        return Topology(gpus, lt, hops, wt, "rocm_smi")
    finally:
        lib.rsmi_shut_down()


def _from_sysfs() -> Optional[Topology]:
    nodes = []
    for d in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*")):
        try:
            props = dict(line.split() for line in open(os.path.join(d, "properties")) if line.strip())
        except OSError:
            continue
        if int(props.get("simd_count", "0")) <= 0:
            continue
        nodes.append((d, props))
    if not nodes:
        return None
    gpus = []
    for i, (_, p) in enumerate(nodes):
        loc = int(p.get("location_id", "0"))
        bdf = "%04x:%02x:%02x.%x" % (int(p.get("domain", "0")), (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 0x7) \
            if loc else ""
        cpus = numa_cpus(bdf) if bdf else []
        gpus.append(GPU(i, bdf, int(p.get("numa_node", "-1")) if "numa_node" in p else -1, cpus))
    N = len(gpus)
    ids = {int(os.path.basename(d)): i for i, (d, _) in enumerate(nodes)}
    lt = [["self" if a == b else "undefined" for b in range(N)] for a in range(N)]
    hops = [[0] * N for _ in range(N)]
    wt = [[0] * N for _ in range(N)]
    for a, (d, _) in enumerate(nodes):
        for link in glob.glob(os.path.join(d, "io_links", "*", "properties")):
            try:
                lp = dict(line.split() for line in open(link) if line.strip())
            except OSError:
                continue
            to = int(lp.get("node_to", "-1"))
            if to not in ids:
                continue
            b = ids[to]
            t = int(lp.get("type", "0"))
            lt[a][b] = "xgmi" if t == 11 else ("pcie" if t == 2 else str(t))
            hops[a][b] = 1
            wt[a][b] = int(lp.get("weight", "0"))
    return Topology(gpus, lt, hops, wt, "sysfs")


def gpu_topology() -> Topology:
    t = _from_rsmi() or _from_sysfs()
    if t is None:
        return Topology([], [], [], [], "none")
    return t


def pin_to_gpu(local_rank: int, topo: Optional[Topology] = None) -> List[int]:
    """Restrict this process to the NUMA-local CPUs of its GPU (no-op if unknown)."""
    # KFD sysfs is a handful of small reads; rocm_smi init costs ~0.2 s per rank
    topo = topo or _from_sysfs()
    if topo is None:
        return []
    visible = os.environ.get("HIP_VISIBLE_DEVICES")
    phys = local_rank
    if visible:
        ids = [int(x) for x in visible.split(",") if x.strip().isdigit()]
        if local_rank < len(ids):
            phys = ids[local_rank]
    if phys >= topo.n:
        return []
    cpus = topo.gpus[phys].cpus
    if not cpus or os.environ.get("PDO_PIN_CPUS", "1") == "0":
        return []
    # only within what this process may already use (a container / cgroup cpuset
    # narrower than the NUMA node): never pin a rank's launch thread onto a
    # handful of CPUs it then shares with the HIP runtime's own threads
    allowed = os.sched_getaffinity(0)
    use = [c for c in cpus if c in allowed]
    if len(use) < min(_MIN_PIN_CPUS, len(allowed)):
        return []
    try:
        os.sched_setaffinity(0, use)
    except OSError:
        return []
    return use


_MIN_PIN_CPUS = 4


def gpu_count() -> int:
    """GPUs this process may use, from KFD sysfs — never initialises HIP.

    Same rule as ``pdo-manager``'s ``detect_gpus`` (csrc/manager/main.cpp): count
    KFD topology nodes with SIMDs, then cap by any visible-devices list.  Safe
    in a process that later fork+execs rank processes (the agent)."""
    n = 0
    for d in glob.glob("/sys/class/kfd/kfd/topology/nodes/*"):
        try:
            with open(os.path.join(d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count":
                        n += int(v) > 0
                        break
        except (OSError, ValueError):
            continue
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def bucket_bytes_for(world: int, grad_bytes: int, links_per_gpu: int = 7) -> int:
    """All-reduce bucket size for the flat-arena DDP (parallel/ddp.py).

    A heuristic from the xGMI link model, NOT a measured knee:
    a ring all-reduce splits each bucket into ``world`` chunks per channel and
    RCCL runs up to ``links_per_gpu`` channels, so ``world × links × 1 MiB``
    keeps ≥ 1 MiB per (ring step × channel) — the regime where a step is
    bandwidth- rather than latency-bound.  Clamped to [16, 256] MiB, and to a
    quarter of the gradient so at least four buckets overlap the backward.
    At world 1 there is nothing to reduce: one bucket.  Pinned by
    tests/test_ddp.py::test_bucket_policy; the 1-GPU RCCL size sweep is
    ``bin/pdo-allreduce-bench`` (profiles/rccl_allreduce_1gpu_r2.md).

    Tuning source: every multi-GPU ``bench.py --gpus N`` record carries
    ``comm.allreduce_sweep`` (busbw of the job's own communicator at 4-256 MiB,
    slowest rank) and ``comm.knee_bytes`` (the smallest size within 90 % of the
    best busbw), next to ``comm.buckets`` (what this policy chose) and
    ``comm.exposed_ms``.  Once a driver SCALE record exists, the per-world
    bucket is set to that ``knee_bytes`` (still capped at a quarter of the
    gradient); until then this stays the link-model heuristic."""
    if world <= 1:
        return max(grad_bytes, 1 << 20)
    b = (1 << 20) * world * links_per_gpu
    b = max(b, 16 << 20)
    b = min(b, 256 << 20, max(grad_bytes // 4, 16 << 20))
    return int(b)


if __name__ == "__main__":
    print(json.dumps(gpu_topology().to_dict(), indent=1))
