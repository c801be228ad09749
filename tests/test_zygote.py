"""Warm-launcher (zygote) slot policies on CPU, with fake slots
(``PDO_SLOT_TEST``): a request parked behind a slot that never becomes ready is
cold-forked after ``PDO_SLOT_PARK_S``; a slot warming past
``PDO_SLOT_WARM_MAX_S`` is killed and counted; ``PDO_SLOT_RESPAWN=exit`` forks
the replacement slot only when the rank that took the warm one exits."""
import os
import socket
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from paddle_operator_amd.launch import zygote  # noqa: E402


def _start(tmp_path, **env):
    path = str(tmp_path / "z.sock")
    e = dict(os.environ, PYTHONPATH=REPO, **env)
    p = subprocess.Popen([sys.executable, "-m", "paddle_operator_amd.launch.zygote", "--socket", path,
                          "--warm-devices", "0"], env=e, stdout=open(tmp_path / "z.log", "w"),
                         stderr=subprocess.STDOUT)
    t_end = time.time() + 120
    while time.time() < t_end and zygote.query_status(path) is None:
        assert p.poll() is None, (tmp_path / "z.log").read_text()
        time.sleep(0.05)
    return p, path, e


def _request(path, env, argv, **extra):
    """Send a launch request the way bin/pdo-launch does; returns the socket
    once the zygote answered PID (or raises on timeout)."""
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(10)
    s.connect(path)
    null = os.open(os.devnull, os.O_RDWR)
    try:
        renv = {k: v for k, v in env.items() if k != "PDO_SLOT_TEST"}
        renv.update({"HIP_VISIBLE_DEVICES": "0"}, **extra)
        req = {"argv": argv, "env": renv,
               "cwd": REPO, "t_start": time.time()}
        zygote._send_request(s, req, [null, null, null])
    finally:
        os.close(null)
    return s


def _readline(s):
    buf = b""
    while not buf.endswith(b"\n"):
        c = s.recv(1)
        if not c:
            break
        buf += c
    return buf.decode()


def _stop(p):
    p.terminate()
    try:
        p.wait(30)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()


def test_parked_request_cold_forks_after_deadline(tmp_path):
    p, path, env = _start(tmp_path, PDO_SLOT_TEST="hang", PDO_SLOT_PARK_S="0.5", PDO_SLOT_WARM_MAX_S="600")
    try:
        st = zygote.query_status(path)
        assert st["slots"]["0"]["ready"] is False
        t0 = time.time()
        s = _request(path, env, ["--workload", "noop", "--exit-after-ready"])
        line = _readline(s)
        waited = time.time() - t0
        assert line.startswith("PID "), line
        assert 0.4 < waited < 5.0, waited
        exit_line = _readline(s)
        assert exit_line.startswith("EXIT "), exit_line
        s.close()
        st = zygote.query_status(path)
        assert st["served"]["park_timeouts"] == 1 and st["served"]["cold"] == 1
        assert st["slots"]["0"]["ready"] is False  # the stuck slot is left to its own deadline
    finally:
        _stop(p)


def test_slot_stuck_warming_is_killed_and_counted(tmp_path):
    p, path, _ = _start(tmp_path, PDO_SLOT_TEST="hang", PDO_SLOT_WARM_MAX_S="0.6")
    try:
        t_end = time.time() + 30
        st = None
        while time.time() < t_end:
            st = zygote.query_status(path)
            if st and st["failed"].get("0", 0) >= zygote.SLOT_RETRIES:
                break
            time.sleep(0.1)
        # every retry got stuck too: killed SLOT_RETRIES times, then no more slots
        assert st["failed"]["0"] >= zygote.SLOT_RETRIES, st
        assert st["served"]["warm_timeouts"] >= zygote.SLOT_RETRIES
        # slots spawned before the retry budget ran out (the pool holds up to
        # slots_per_gpu) hit their own deadline; none is respawned after that
        t_end = time.time() + 30
        while time.time() < t_end and "0" in zygote.query_status(path)["slots"]:
            time.sleep(0.1)
        assert "0" not in zygote.query_status(path)["slots"]
        n_failed = zygote.query_status(path)["failed"]["0"]
        time.sleep(1.5)  # > PDO_SLOT_WARM_MAX_S: a respawned slot would have failed again by now
        st = zygote.query_status(path)
        assert "0" not in st["slots"] and st["failed"]["0"] == n_failed, st
    finally:
        _stop(p)


@pytest.mark.parametrize("policy", ["handoff", "exit"])
def test_slot_respawn_policy(tmp_path, policy):
    p, path, env = _start(tmp_path, PDO_SLOT_TEST="cpu", PDO_SLOT_RESPAWN=policy, PDO_SLOTS_PER_GPU="1")
    try:
        t_end = time.time() + 30
        while time.time() < t_end and not (zygote.query_status(path)["slots"].get("0") or {}).get("ready"):
            time.sleep(0.05)
        # the rank (the slot itself, now running the request) stays alive 1.5 s
        s = _request(path, env, ["--workload", "noop", "--exit-after-ready"], PDO_RANK_HOLD_S="1.5")
        assert _readline(s).startswith("PID ")
        time.sleep(0.5)
        st = zygote.query_status(path)
        assert st["served"]["warm"] == 1 and st["respawn"] == policy
        if policy == "handoff":
            assert "0" in st["slots"]  # replacement forked at handoff, beside the running job
        else:
            assert "0" not in st["slots"]  # no second process on the GPU while the job runs
        assert _readline(s).startswith("EXIT ")
        t_exit = time.time()
        s.close()
        t_end = time.time() + 30
        while time.time() < t_end and "0" not in zygote.query_status(path)["slots"]:
            time.sleep(0.05)
        st = zygote.query_status(path)
        assert "0" in st["slots"]  # respawned either way once the rank exited
        if policy == "exit":
            assert st["slots"]["0"]["t_spawn"] > t_exit - 1.0
    finally:
        _stop(p)


def test_two_slots_serve_back_to_back_jobs_warm(tmp_path):
    """PDO_SLOTS_PER_GPU=2: a job arriving while the first job's replacement
    slot is still warming takes the second warm slot instead of parking."""
    p, path, env = _start(tmp_path, PDO_SLOT_TEST="cpu", PDO_SLOTS_PER_GPU="2")
    try:
        t_end = time.time() + 30
        while time.time() < t_end:
            sl = zygote.query_status(path)["slots"].get("0") or {}
            if sl.get("n_ready") == 2:
                break
            time.sleep(0.05)
        st = zygote.query_status(path)
        assert st["slots_per_gpu"] == 2 and st["slots"]["0"]["n_ready"] == 2, st
        socks = []
        for _ in range(2):  # back to back: no wait for the replacement
            s = _request(path, env, ["--workload", "noop", "--exit-after-ready"], PDO_RANK_HOLD_S="1.0")
            assert _readline(s).startswith("PID ")
            socks.append(s)
        st = zygote.query_status(path)
        assert st["served"]["warm"] == 2 and st["served"]["cold"] == 0, st
        assert st["served"]["park_timeouts"] == 0
        for s in socks:
            assert _readline(s).startswith("EXIT ")
            s.close()
    finally:
        _stop(p)


def test_back_to_back_stream_dispatch_delay_bounded(tmp_path):
    """A stream of back-to-back jobs on one GPU while replacement slots warm
    (simulated 1.0 s warm-up, one job every ≈ 0.45 s — the round-5 b2b regime
    scaled down): with the default pool (3 slots at ≤ 2 GPUs) no request parks
    long; the zygote's own stamps (PDO_T_ZYG_RECV / PDO_T_DISPATCH) bound it."""
    env0 = {k: v for k, v in os.environ.items() if k != "PDO_SLOTS_PER_GPU"}
    path = str(tmp_path / "z.sock")
    e = dict(env0, PYTHONPATH=REPO, PDO_SLOT_TEST="cpu", PDO_SLOT_TEST_WARM_S="1.0")
    p = subprocess.Popen([sys.executable, "-m", "paddle_operator_amd.launch.zygote", "--socket", path,
                          "--warm-devices", "0"], env=e, stdout=open(tmp_path / "z.log", "w"),
                         stderr=subprocess.STDOUT)
    try:
        t_end = time.time() + 120
        st = None
        while time.time() < t_end:
            st = zygote.query_status(path)
            if st and (st["slots"].get("0") or {}).get("n_ready") == st["slots_per_gpu"]:
                break
            time.sleep(0.05)
        assert st["slots_per_gpu"] == 3, st
        for _ in range(7):
            t0 = time.time()
            s = _request(path, e, ["--workload", "noop", "--exit-after-ready"], PDO_RANK_HOLD_S="0.1")
            assert _readline(s).startswith("PID ")
            assert _readline(s).startswith("EXIT ")
            s.close()
            time.sleep(max(0.0, 0.45 - (time.time() - t0)))
        st = zygote.query_status(path)
        assert st["served"]["warm"] == 7 and st["served"]["cold"] == 0, st
        # every request dispatched at once: nothing parked behind a warming slot
        assert st["served"]["park_max_s"] < 0.1, st["served"]
    finally:
        _stop(p)


def test_two_slot_pool_parks_under_the_same_stream(tmp_path):
    """The same stream with PDO_SLOTS_PER_GPU=2 parks (the round-5 regression's
    mechanism): warm_s / 2 > the job interval."""
    p, path, env = _start(tmp_path, PDO_SLOT_TEST="cpu", PDO_SLOT_TEST_WARM_S="1.0", PDO_SLOTS_PER_GPU="2")
    try:
        t_end = time.time() + 60
        while time.time() < t_end and (zygote.query_status(path)["slots"].get("0") or {}).get("n_ready") != 2:
            time.sleep(0.05)
        for _ in range(6):
            t0 = time.time()
            s = _request(path, env, ["--workload", "noop", "--exit-after-ready"], PDO_RANK_HOLD_S="0.1")
            assert _readline(s).startswith("PID ")
            assert _readline(s).startswith("EXIT ")
            s.close()
            time.sleep(max(0.0, 0.3 - (time.time() - t0)))
        st = zygote.query_status(path)
        assert st["served"]["parked"] >= 1 and st["served"]["park_max_s"] > 0.1, st["served"]
    finally:
        _stop(p)
