"""Warm launcher ("zygote") — fork pre-imported rank processes.

Python start-up plus ``import torch`` costs ≈1.2–1.5 s per rank, the largest
single term of job-start → ready once the control plane is event-driven.  A
per-node zygote imports torch and the pdo modules ONCE (without touching the
GPU runtime: no HIP call happens before fork, so every child initialises HIP
itself after ``HIP_VISIBLE_DEVICES`` is set) and forks a rank on request.

The native client ``bin/pdo-launch`` (csrc/agent/launch_client.cpp) is the
container's entry point: with ``PDO_ZYGOTE=<unix socket>`` reachable it sends
``{argv, env, cwd, t_start}`` plus its stdin/stdout/stderr fds
(SCM_RIGHTS), prints nothing itself, relays signals to the child and exits
with the child's status — so the kubelet-lite agent still tracks one process
per container with its real exit code.  Without a zygote it execs
``python -m paddle_operator_amd.launch`` (cold path).

Protocol (SOCK_STREAM): client → u32 length + JSON (fds attached);
server → ``PID <pid>\\n`` then ``EXIT <status>\\n`` (status = exit code, or
128+signal).  EOF from the client (it was SIGKILLed) kills the child's
process group.  The server is single-threaded (selector loop + WNOHANG
reaping) so ``fork`` never happens with other Python threads alive.

GPU-warm slots (``--warm-devices 0,1,…``, one per node GPU, passed by the
agent): the import saving leaves HIP init (≈0.15 s) and RCCL communicator
init (≈1.1 s, almost all of it RCCL loading its device code objects into the
new process — profiles/r2_launched_bench_1gpu.md) inside every rank.  A slot is
forked from the zygote BEFORE any HIP call, binds one GPU
(``HIP_VISIBLE_DEVICES``), initialises HIP, builds and destroys a 1-rank RCCL
communicator (kernels now resident) and then blocks on its socketpair.  A
request for exactly that GPU, whose runtime-relevant environment (HIP_/HSA_/
ROCR_/GPU_/NCCL_/RCCL_/PYTORCH_/TORCH_/AMD_/LD_ variables — read once per
process by HIP/RCCL/torch) equals the slot's, is handed to the slot (request +
client fds over the socketpair) instead of forking: the slot BECOMES the rank
and builds the job's real communicator (world size, rendezvous, rings) from
scratch — only the process-level warm-up is reused.  A replacement slot for
that GPU is forked at once and warms while the job runs.  Requests that could
exec (elastic agents spawn their workers) or that differ in those variables
take the cold fork.  ``PDO_WARM_SLOT=0`` in a pod's env opts it out.
"""
from __future__ import annotations

import array
import json
import os
import selectors
import signal
import socket
import struct
import sys
import time
from typing import Dict, List, Optional

PRELOAD = (
    "torch", "torch.distributed", "torch.nn.functional", "numpy",
    "paddle_operator_amd.launch.run", "paddle_operator_amd.launch.bootstrap", "paddle_operator_amd.launch.env",
    "paddle_operator_amd.launch.elastic", "paddle_operator_amd.kv.client", "paddle_operator_amd.utils.checkpoint",
    "paddle_operator_amd.utils.topology", "paddle_operator_amd.models.gpt2", "paddle_operator_amd.models.resnet",
    "paddle_operator_amd.models.wide_deep", "paddle_operator_amd.parallel.flat", "paddle_operator_amd.parallel.ddp",
    "paddle_operator_amd.workloads.resnet", "paddle_operator_amd.train", "paddle_operator_amd.ops",
    "paddle_operator_amd.ops.optim",
)


def preload():
    import importlib
    t0 = time.time()
    for m in PRELOAD:
        try:
            importlib.import_module(m)
        except Exception as e:  # a missing optional module must not stop the zygote
            print(f"[pdo-zygote] preload {m} failed: {e}", file=sys.stderr, flush=True)
    return time.time() - t0


# variables HIP / RCCL / torch read once per process: a warm slot initialised
# under one set of them cannot serve a request asking for another
WARM_PREFIXES = ("HIP_", "HSA_", "ROCR_", "GPU_", "NCCL_", "RCCL_", "PYTORCH_", "TORCH_", "AMD_", "LD_", "CUDA_")
WARM_IGNORE = ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
SLOT_RETRIES = 3
# a request parked behind a still-warming slot is cold-forked after this long
# (≈ the cold start it was parked to avoid): a slot stuck in HIP or RCCL init
# must never hold a pod's launch hostage (PDO_SLOT_PARK_S)
SLOT_PARK_S = float(os.environ.get("PDO_SLOT_PARK_S", "2.5"))
# a slot still warming after this long is killed and counted as a failure
SLOT_WARM_MAX_S = float(os.environ.get("PDO_SLOT_WARM_MAX_S", "60"))
# when the replacement slot for a GPU is forked: "handoff" = as soon as a job
# takes the warm slot (the next job on that GPU starts warm; the replacement's
# HIP context and 1-rank communicator stay resident beside the job, see
# "mem_mb" in the status table), "exit" = once that job's rank exits (no
# second context on the GPU while the job runs)
SLOT_RESPAWN = os.environ.get("PDO_SLOT_RESPAWN", "handoff")
# warm slots kept per GPU (PDO_SLOTS_PER_GPU).  A slot re-warms in ≈ 1.6 s (HIP
# + RCCL init, 'warm_s' in the status table) while back-to-back jobs on one GPU
# arrive every ≈ 0.7 s (bench.py 'ready_b2b': create → ready → Completed →
# deleted).  A pool of k slots absorbs such a stream only while warm_s / k ≤
# the job interval: with two, every job from the third on parked ≈ 1.6 − 2·0.7
# ≈ 0.2 s behind a warming slot (the round-5 'ready_b2b' p50 of 0.27 s, entry
# phase 0.20 s); three keep it at zero.  Each slot holds a HIP context and a
# 1-rank communicator on the GPU ('mem_mb' ≈ 1 GB of the 288 GB).  Unset, the
# default follows the number of warm devices (slots_per_gpu): three up to 2
# GPUs, one above, so a full 8-GPU node runs at most rank + slot = 2 processes
# per GPU — the layout bench.py measures.
_SLOTS_ENV = os.environ.get("PDO_SLOTS_PER_GPU", "")


def slots_per_gpu(n_devices: int) -> int:
    if _SLOTS_ENV.strip():
        return max(1, int(_SLOTS_ENV))
    return 3 if n_devices <= 2 else 1


SLOTS_PER_GPU = slots_per_gpu(1)


def runtime_key(env: Dict[str, str]) -> tuple:
    return tuple(sorted((k, v) for k, v in env.items() if k.startswith(WARM_PREFIXES) and k not in WARM_IGNORE))


def warm_device_of(req: dict, key: tuple) -> Optional[str]:
    """The GPU id a request may take a warm slot for, or None (cold fork)."""
    env = req.get("env") or {}
    argv = req.get("argv") or []
    dev = env.get("HIP_VISIBLE_DEVICES", "") or env.get("PDO_GPU_IDS", "")
    if not dev or "," in dev or env.get("PDO_WARM_SLOT", "1") == "0":
        return None
    # elastic agents fork+exec their workers: never from a HIP-initialised process
    if "--elastic" in argv or "--worker" in argv or env.get("PADDLE_ELASTIC_JOB_ID") or env.get("PADDLE_ELASTIC_NP"):
        return None
    # a pod supervising several local ranks forks them: never from a warm slot
    if "--nproc-per-pod" in argv or int(env.get("PDO_NPROC_PER_POD", "1") or 1) > 1:
        return None
    return dev if runtime_key(env) == key else None


def _send_request(sock: socket.socket, req: dict, fds: List[int]):
    body = json.dumps(req).encode()
    anc = [(socket.SOL_SOCKET, socket.SCM_RIGHTS, array.array("i", fds).tobytes())] if fds else []
    sock.sendmsg([struct.pack("<I", len(body))], anc)
    sock.sendall(body)


def _recv_request(conn: socket.socket):
    fds = array.array("i")
    hdr, anc, _, _ = conn.recvmsg(4, socket.CMSG_SPACE(8 * fds.itemsize))
    for level, typ, data in anc:
        if level == socket.SOL_SOCKET and typ == socket.SCM_RIGHTS:
            fds.frombytes(data[:len(data) - len(data) % fds.itemsize])
    if len(hdr) < 4:
        raise EOFError("short header")
    (n,) = struct.unpack("<I", hdr)
    buf = b""
    while len(buf) < n:
        chunk = conn.recv(n - len(buf))
        if not chunk:
            raise EOFError("short body")
        buf += chunk
    return json.loads(buf), list(fds)


def _child(req, fds, listener):
    """In the forked child: become the rank process and never return."""
    try:
        listener.close()
        os.setsid()
    except BaseException:
        os._exit(1)
    _become_rank(req, fds)


def _become_rank(req, fds, warm=False):
    rc = 1
    try:
        for target, fd in zip((0, 1, 2), fds):
            os.dup2(fd, target)
        if warm:
            # a warm slot closed the zygote's descriptors before HIP init; what it
            # holds now is the HIP runtime's (/dev/kfd, render node, ...)
            for fd in fds:
                if fd > 2:
                    os.close(fd)
        else:
            # nothing of the zygote's survives into the rank: its selector, the other
            # clients' connections and the passed originals (0-2 now hold the client's)
            os.closerange(3, 65536)
        signal.signal(signal.SIGTERM, signal.SIG_DFL)
        signal.signal(signal.SIGINT, signal.default_int_handler)
        signal.signal(signal.SIGCHLD, signal.SIG_DFL)
        os.chdir(req.get("cwd") or "/")
        os.environ.clear()
        os.environ.update(req.get("env") or {})
        # torch sized its intra-op pool when the ZYGOTE imported it (its
        # environment, typically every CPU); the pod's OMP_NUM_THREADS must still
        # hold in the rank — 8 forked CPU ranks on 8 CPUs each ran 8 spinning
        # OpenMP threads: 16 s per tiny ResNet step instead of 10 ms
        omp = (os.environ.get("OMP_NUM_THREADS") or "").strip()
        if omp.isdigit() and int(omp) > 0 and "torch" in sys.modules:
            sys.modules["torch"].set_num_threads(int(omp))
        argv = list(req.get("argv") or [])
        sys.argv = ["pdo-launch"] + argv
        sys.stdout = os.fdopen(1, "w", buffering=1, closefd=False)
        sys.stderr = os.fdopen(2, "w", buffering=1, closefd=False)
        hold = float(os.environ.get("PDO_RANK_HOLD_S", "0") or 0)
        if hold > 0:  # tests: a rank that stays alive this long before it runs
            time.sleep(hold)
        from paddle_operator_amd.launch import run
        run.T_START = float(req.get("t_start") or time.time())
        rc = int(run.main(argv) or 0)
    except SystemExit as e:
        rc = e.code if isinstance(e.code, int) else (0 if e.code is None else 1)
    except BaseException:
        import traceback
        traceback.print_exc()
        rc = 1
    finally:
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:
            pass
        os._exit(rc)


def _warm_gpu(index: int = 0) -> dict:
    """HIP init + a 1-rank RCCL communicator built and destroyed (loads RCCL's
    device code into this process) on device ``index``: 0 = the slot's one
    visible GPU, or the GPU's own index when every GPU is visible
    (PDO_GPU_VISIBILITY=all)."""
    import torch
    import torch.distributed as dist

    from ..utils import topology
    t0 = time.time()
    topology.pin_to_gpu(index)
    if not torch.cuda.is_available():  # a GPU node with no usable HIP device: nothing to warm
        return {"device": "none"}
    torch.cuda.set_device(index)
    torch.cuda.init()
    dev = torch.device("cuda", index)
    free0, total = torch.cuda.mem_get_info(dev)
    t1 = time.time()
    dist.init_process_group("nccl", rank=0, world_size=1, store=dist.HashStore(), device_id=dev)
    t = torch.ones(1, device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize(dev)
    dist.destroy_process_group()
    del t
    free1, _ = torch.cuda.mem_get_info(dev)
    # device memory this warm process holds while it waits (HIP context + RCCL
    # code objects); mem_get_info is device-wide, so this is an upper bound
    # when other processes allocate on the GPU meanwhile
    return {"hip_s": round(t1 - t0, 4), "rccl_s": round(time.time() - t1, 4),
            "mem_mb": round((total - free1) / 2**20, 1), "mem_mb_before_rccl": round((total - free0) / 2**20, 1)}


def _slot_main(dev: str, sock: socket.socket, listener: socket.socket):
    """A forked GPU-warm slot: warm up, report READY, wait for one request,
    become that rank.  Never returns."""
    try:
        listener.close()
        os.setsid()
        keep = sock.fileno()
        os.closerange(3, keep)
        os.closerange(keep + 1, 65536)
        for sig in (signal.SIGTERM, signal.SIGCHLD):
            signal.signal(sig, signal.SIG_DFL)
        os.environ.pop("CUDA_VISIBLE_DEVICES", None)
        test_mode = os.environ.get("PDO_SLOT_TEST", "")
        if test_mode == "hang":  # CPU tests: a slot stuck in its warm-up
            while True:
                time.sleep(3600)
        if test_mode == "cpu":  # CPU tests: a slot that warms nothing (in PDO_SLOT_TEST_WARM_S)
            time.sleep(float(os.environ.get("PDO_SLOT_TEST_WARM_S", "0") or 0))
            info = {"device": "none"}
        elif os.environ.get("PDO_GPU_VISIBILITY") == "all":
            os.environ.pop("HIP_VISIBLE_DEVICES", None)
            info = _warm_gpu(int(dev))
        else:
            os.environ["HIP_VISIBLE_DEVICES"] = dev
            info = _warm_gpu()
        info["pid"] = os.getpid()
        sock.sendall(f"READY {json.dumps(info)}\n".encode())
        req, fds = _recv_request(sock)
    except EOFError:  # the zygote is shutting down
        os._exit(0)
    except BaseException as e:
        try:
            sock.sendall(f"FAIL {type(e).__name__}: {e}\n".encode())
        except OSError:
            pass
        os._exit(3)
    sock.close()
    req.setdefault("env", {})["PDO_WARM_SLOT_USED"] = "1"
    _become_rank(req, fds, warm=True)


class _Slot:
    def __init__(self, dev, pid, sock):
        self.dev, self.pid, self.sock = dev, pid, sock
        self.ready = False
        self.t_spawn = time.time()
        self.info: dict = {}


def serve(path: str, idle_exit_s: float = 0.0, warm_devices: Optional[List[str]] = None):
    took = preload()
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
    ls = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    ls.bind(path)
    os.chmod(path, 0o600)
    ls.listen(256)
    ls.setblocking(False)
    print(f"[pdo-zygote] ready on {path} (preload {took:.2f}s, pid {os.getpid()})", flush=True)
    sel = selectors.DefaultSelector()
    sel.register(ls, selectors.EVENT_READ, "listen")
    children = {}  # pid -> conn
    stop = []
    signal.signal(signal.SIGTERM, lambda *a: stop.append(1))
    last_activity = time.time()
    key = runtime_key(dict(os.environ))
    slots: Dict[str, List[_Slot]] = {}  # device -> its warm slots (≤ per_gpu)
    slot_pids: Dict[int, _Slot] = {}
    slot_fails: Dict[str, int] = {}
    pending: Dict[str, list] = {}      # device -> [(conn, req, fds, t_park)] waiting for a warming slot
    rank_dev: Dict[int, str] = {}      # rank pid -> GPU whose slot it took (SLOT_RESPAWN = exit)
    served = {"warm": 0, "cold": 0, "park_timeouts": 0, "warm_timeouts": 0, "parked": 0, "park_s": 0.0,
              "park_max_s": 0.0}
    per_gpu = slots_per_gpu(len(warm_devices or ()))

    def log(msg):
        print(f"[pdo-zygote] {msg}", flush=True)

    def ready_slot(dev):
        return next((s for s in slots.get(dev, ()) if s.ready), None)

    def spawn_slot(dev):
        if stop or slot_fails.get(dev, 0) >= SLOT_RETRIES or len(slots.get(dev, ())) >= per_gpu:
            return
        a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
        pid = os.fork()
        if pid == 0:
            a.close()
            _slot_main(dev, b, ls)
        b.close()
        sl = _Slot(dev, pid, a)
        slots.setdefault(dev, []).append(sl)
        slot_pids[pid] = sl
        sel.register(a, selectors.EVENT_READ, ("slot", sl))

    def drop_slot(sl):
        lst = slots.get(sl.dev)
        if lst and sl in lst:
            lst.remove(sl)
            if not lst:
                slots.pop(sl.dev)
        try:
            sel.unregister(sl.sock)
        except (KeyError, ValueError):
            pass
        sl.sock.close()

    def attach(pid, conn):
        children[pid] = conn
        try:
            conn.sendall(f"PID {pid}\n".encode())
        except OSError:
            pass
        conn.setblocking(False)
        sel.register(conn, selectors.EVENT_READ, pid)

    def stamp(req, how):
        """Dispatch timestamps for the rank's phase split (launch/bootstrap.py):
        request received → handed to a slot / forked; parked time is counted."""
        now = time.time()
        env = req.setdefault("env", {})
        t_recv = float(req.get("_t_recv") or now)
        env["PDO_T_ZYG_RECV"] = repr(t_recv)
        env["PDO_T_DISPATCH"] = repr(now)
        env["PDO_DISPATCH"] = how
        served["park_s"] = round(served["park_s"] + (now - t_recv), 4)
        served["park_max_s"] = round(max(served["park_max_s"], now - t_recv), 4)

    def cold(conn, req, fds):
        stamp(req, "cold")
        pid = os.fork()
        if pid == 0:
            _child(req, fds, ls)
        for fd in fds:
            os.close(fd)
        served["cold"] += 1
        attach(pid, conn)

    def handoff(sl, conn, req, fds):
        stamp(req, "warm")
        try:
            _send_request(sl.sock, req, fds)
        except OSError as e:  # the slot died under us
            log(f"slot {sl.dev} pid {sl.pid} handoff failed ({e}); cold fork")
            drop_slot(sl)
            cold(conn, req, fds)
            return
        for fd in fds:
            os.close(fd)
        drop_slot(sl)
        slot_pids.pop(sl.pid, None)
        served["warm"] += 1
        attach(sl.pid, conn)
        if SLOT_RESPAWN == "exit":
            rank_dev[sl.pid] = sl.dev  # the replacement is forked when this rank exits
        else:
            spawn_slot(sl.dev)  # the replacement warms while this job runs

    def flush_pending(dev):
        for conn, req, fds, _ in pending.pop(dev, []):
            sl = ready_slot(dev)
            if sl is not None:
                handoff(sl, conn, req, fds)
            else:
                cold(conn, req, fds)

    def expire(now):
        """Cold-fork requests parked past SLOT_PARK_S; kill slots warming past
        SLOT_WARM_MAX_S (counted in slot_fails; the reaper respawns up to
        SLOT_RETRIES)."""
        for dev in list(pending):
            keep = []
            for ent in pending[dev]:
                if now - ent[3] > SLOT_PARK_S:
                    served["park_timeouts"] += 1
                    log(f"request parked {now - ent[3]:.1f}s behind warming slot gpu {dev}; cold fork")
                    cold(*ent[:3])
                else:
                    keep.append(ent)
            if keep:
                pending[dev] = keep
            else:
                pending.pop(dev)
        for sl in [x for lst in slots.values() for x in lst]:
            if not sl.ready and now - sl.t_spawn > SLOT_WARM_MAX_S:
                served["warm_timeouts"] += 1
                log(f"slot gpu {sl.dev} pid {sl.pid} still warming after {now - sl.t_spawn:.0f}s; killed")
                slot_fails[sl.dev] = slot_fails.get(sl.dev, 0) + 1
                try:
                    os.killpg(sl.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                drop_slot(sl)
                flush_pending(sl.dev)

    def status_table():
        # a slot still warming reports its GPU's last READY record (footprint,
        # warm time), so a status read right after a handoff is not empty
        def one(d, lst):  # a ready slot first; n / n_ready count the pool
            sl = next((x for x in lst if x.ready), lst[0])
            return {"pid": sl.pid, "ready": sl.ready, "t_spawn": max(x.t_spawn for x in lst), "n": len(lst),
                    "n_ready": sum(x.ready for x in lst), **(sl.info or last_info.get(d, {}))}
        return {"pid": os.getpid(), "served": served,
                "slots": {d: one(d, lst) for d, lst in slots.items() if lst},
                "slots_per_gpu": per_gpu,
                "respawn": SLOT_RESPAWN, "park_s": SLOT_PARK_S,
                "devices": list(warm_devices or []), "failed": slot_fails}

    last_info = {}
    for dev in warm_devices or []:
        for _ in range(per_gpu):
            spawn_slot(dev)
    while not stop:
        for skey, _ in sel.select(timeout=0.01):
            if skey.data == "listen":
                try:
                    conn, _ = ls.accept()
                except BlockingIOError:
                    continue
                conn.setblocking(True)
                try:
                    req, fds = _recv_request(conn)
                except Exception as e:
                    print(f"[pdo-zygote] bad request: {e}", file=sys.stderr, flush=True)
                    conn.close()
                    continue
                if req.get("op") == "status":
                    try:
                        conn.sendall(f"STATUS {json.dumps(status_table())}\n".encode())
                    except OSError:
                        pass
                    conn.close()
                    continue
                last_activity = req["_t_recv"] = time.time()
                dev = warm_device_of(req, key) if warm_devices else None
                sl = ready_slot(dev) if dev is not None else None
                if sl is not None:
                    handoff(sl, conn, req, fds)
                elif dev is not None and slots.get(dev):  # warming: wait for one, at most SLOT_PARK_S (expire)
                    served["parked"] += 1
                    pending.setdefault(dev, []).append((conn, req, fds, time.time()))
                else:
                    cold(conn, req, fds)
            elif isinstance(skey.data, tuple):  # a slot's control socket
                sl = skey.data[1]
                try:
                    line = sl.sock.recv(4096).decode(errors="replace")
                except (BlockingIOError, InterruptedError):
                    continue
                except OSError:
                    line = ""
                if line.startswith("READY"):
                    sl.ready = True
                    try:
                        sl.info = json.loads(line[5:].strip() or "{}")
                    except ValueError:
                        sl.info = {}
                    sl.info["warm_s"] = round(time.time() - sl.t_spawn, 3)
                    last_info[sl.dev] = dict(sl.info)
                    slot_fails.pop(sl.dev, None)
                    log(f"slot gpu {sl.dev} warm in {sl.info['warm_s']}s ({sl.info})")
                    flush_pending(sl.dev)
                else:  # FAIL or EOF: the slot is gone; its pid is reaped below
                    log(f"slot gpu {sl.dev} pid {sl.pid} failed: {line.strip() or 'EOF'}")
                    slot_fails[sl.dev] = slot_fails.get(sl.dev, 0) + 1
                    drop_slot(sl)
                    flush_pending(sl.dev)
            else:
                pid, conn = skey.data, skey.fileobj
                try:
                    data = conn.recv(64)
                except (BlockingIOError, InterruptedError):
                    continue
                except OSError:
                    data = b""
                if not data:  # client gone (SIGKILL): take the rank down with it
                    sel.unregister(conn)
                    try:
                        os.killpg(pid, signal.SIGKILL)
                    except (ProcessLookupError, PermissionError):
                        pass
        expire(time.time())
        # reap
        while children or slot_pids:
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                break
            if pid == 0:
                break
            sl = slot_pids.pop(pid, None)
            if sl is not None:  # an unused slot exited
                if sl in slots.get(sl.dev, ()):
                    slot_fails[sl.dev] = slot_fails.get(sl.dev, 0) + 1
                    drop_slot(sl)
                    flush_pending(sl.dev)
                spawn_slot(sl.dev)
                continue
            conn = children.pop(pid, None)
            if pid in rank_dev:
                spawn_slot(rank_dev.pop(pid))
            code = os.waitstatus_to_exitcode(status)
            code = 128 - code if code < 0 else code
            if conn is not None:
                try:
                    sel.unregister(conn)
                except (KeyError, ValueError):
                    pass
                try:
                    conn.setblocking(True)
                    conn.sendall(f"EXIT {code}\n".encode())
                except OSError:
                    pass
                conn.close()
            last_activity = time.time()
        if idle_exit_s and not children and time.time() - last_activity > idle_exit_s:
            break
    for pid in list(children):
        try:
            os.killpg(pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
    for sl in [x for lst in slots.values() for x in lst]:  # idle slots exit on EOF
        drop_slot(sl)
    for pid in list(slot_pids):
        try:
            os.waitpid(pid, 0)
        except ChildProcessError:
            pass
    ls.close()
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(prog="pdo-zygote")
    ap.add_argument("--socket", default=os.environ.get("PDO_ZYGOTE", "/tmp/pdo-zygote.sock"))
    ap.add_argument("--idle-exit", type=float, default=0.0)
    ap.add_argument("--warm-devices", default="",
                    help="comma-separated GPU ids (as HIP_VISIBLE_DEVICES values) to keep a warm slot for")
    a = ap.parse_args(argv)
    serve(a.socket, a.idle_exit, [d for d in a.warm_devices.split(",") if d.strip()])


def query_status(path: str, timeout: float = 2.0) -> Optional[dict]:
    """The zygote's slot table (``None`` if it is not reachable)."""
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    try:
        s.connect(path)
        _send_request(s, {"op": "status"}, [])
        buf = b""
        while not buf.endswith(b"\n"):
            chunk = s.recv(65536)
            if not chunk:
                break
            buf += chunk
    except OSError:
        return None
    finally:
        s.close()
    line = buf.decode(errors="replace").strip()
    return json.loads(line[7:]) if line.startswith("STATUS ") else None


if __name__ == "__main__":
    main()
