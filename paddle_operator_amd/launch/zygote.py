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
    rc = 1
    try:
        listener.close()
        os.setsid()
        for target, fd in zip((0, 1, 2), fds):
            os.dup2(fd, target)
        # nothing of the zygote's survives into the rank: its selector, the other
        # clients' connections and the passed originals (0-2 now hold the client's)
        os.closerange(3, 65536)
        signal.signal(signal.SIGTERM, signal.SIG_DFL)
        signal.signal(signal.SIGINT, signal.default_int_handler)
        signal.signal(signal.SIGCHLD, signal.SIG_DFL)
        os.chdir(req.get("cwd") or "/")
        os.environ.clear()
        os.environ.update(req.get("env") or {})
        argv = list(req.get("argv") or [])
        sys.argv = ["pdo-launch"] + argv
        sys.stdout = os.fdopen(1, "w", buffering=1, closefd=False)
        sys.stderr = os.fdopen(2, "w", buffering=1, closefd=False)
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


def serve(path: str, idle_exit_s: float = 0.0):
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
    while not stop:
        for key, _ in sel.select(timeout=0.01):
            if key.data == "listen":
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
                pid = os.fork()
                if pid == 0:
                    _child(req, fds, ls)
                for fd in fds:
                    os.close(fd)
                children[pid] = conn
                try:
                    conn.sendall(f"PID {pid}\n".encode())
                except OSError:
                    pass
                conn.setblocking(False)
                sel.register(conn, selectors.EVENT_READ, pid)
                last_activity = time.time()
            else:
                pid, conn = key.data, key.fileobj
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
        # reap
        while children:
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                break
            if pid == 0:
                break
            conn = children.pop(pid, None)
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
    a = ap.parse_args(argv)
    serve(a.socket, a.idle_exit)


if __name__ == "__main__":
    main()
