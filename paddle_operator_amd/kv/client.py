"""Client for pdo-kv (and any etcd ≥ 3.4 through its JSON gateway).

Used by the launcher for rendezvous (elastic membership, ``np`` key, RCCL
readiness barrier) — the same key layout the reference's elastic mode uses
(``/paddle/<ns>-<name>/np``, controllers/paddlejob_elastic.go:44).
Pure standard library (http.client), base64 keys/values, int64-as-string.
"""
from __future__ import annotations

import base64
import http.client
import json
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple
from urllib.parse import urlparse


def _b64(s) -> str:
    if isinstance(s, str):
        s = s.encode()
    return base64.b64encode(s).decode()


def _unb64(s: Optional[str]) -> str:
    return base64.b64decode(s or "").decode(errors="replace")


def prefix_end(prefix: str) -> str:
    b = bytearray(prefix.encode())
    for i in range(len(b) - 1, -1, -1):
        if b[i] < 0xFF:
            b[i] += 1
            return bytes(b[: i + 1]).decode(errors="surrogateescape")
    return "\0"


class KVError(RuntimeError):
    pass


class KVClient:
    def __init__(self, endpoints: str, timeout: float = 3.0):
        self.endpoints = [e.strip() for e in endpoints.split(",") if e.strip()]
        if not self.endpoints:
            raise ValueError("no kv endpoints")
        self.timeout = timeout

    def _host(self, ep: str) -> Tuple[str, int]:
        if "://" not in ep:
            ep = "http://" + ep
        u = urlparse(ep)
        return u.hostname, u.port or 2379

    def _call(self, path: str, body: dict, timeout: Optional[float] = None) -> dict:
        last = None
        for ep in self.endpoints:
            host, port = self._host(ep)
            try:
                c = http.client.HTTPConnection(host, port, timeout=timeout or self.timeout)
                c.request("POST", path, json.dumps(body), {"Content-Type": "application/json"})
                r = c.getresponse()
                data = r.read()
                c.close()
                if r.status != 200:
                    raise KVError(f"{path}: HTTP {r.status} {data[:200]!r}")
                return json.loads(data or b"{}")
            except (OSError, http.client.HTTPException) as e:
                last = e
        raise KVError(f"kv unreachable ({self.endpoints}): {last}")

    # -- kv -----------------------------------------------------------------
    def get(self, key: str) -> Optional[str]:
        r = self._call("/v3/kv/range", {"key": _b64(key)})
        kvs = r.get("kvs") or []
        return _unb64(kvs[0].get("value")) if kvs else None

    def get_prefix(self, prefix: str) -> Dict[str, str]:
        r = self._call("/v3/kv/range", {"key": _b64(prefix), "range_end": _b64(prefix_end(prefix))})
        return {_unb64(kv["key"]): _unb64(kv.get("value")) for kv in r.get("kvs") or []}

    def put(self, key: str, value: str, lease: int = 0) -> int:
        body = {"key": _b64(key), "value": _b64(value)}
        if lease:
            body["lease"] = str(lease)
        r = self._call("/v3/kv/put", body)
        return int(r.get("header", {}).get("revision", 0))

    def delete(self, key: str, prefix: bool = False) -> int:
        body = {"key": _b64(key)}
        if prefix:
            body["range_end"] = _b64(prefix_end(key))
        return int(self._call("/v3/kv/deleterange", body).get("deleted", 0))

    def put_if_absent(self, key: str, value: str, lease: int = 0) -> bool:
        """Atomic create (txn: version(key) == 0)."""
        put = {"key": _b64(key), "value": _b64(value)}
        if lease:
            put["lease"] = str(lease)
        r = self._call("/v3/kv/txn", {
            "compare": [{"key": _b64(key), "target": "VERSION", "result": "EQUAL", "version": "0"}],
            "success": [{"request_put": put}],
        })
        return bool(r.get("succeeded"))

    def cas(self, key: str, expect: str, value: str) -> bool:
        r = self._call("/v3/kv/txn", {
            "compare": [{"key": _b64(key), "target": "VALUE", "result": "EQUAL", "value": _b64(expect)}],
            "success": [{"request_put": {"key": _b64(key), "value": _b64(value)}}],
        })
        return bool(r.get("succeeded"))

    def revision(self) -> int:
        r = self._call("/v3/kv/range", {"key": _b64("\0"), "count_only": True})
        return int(r.get("header", {}).get("revision", 0))

    # -- leases -------------------------------------------------------------
    def lease_grant(self, ttl: int) -> int:
        return int(self._call("/v3/lease/grant", {"TTL": str(ttl)})["ID"])

    def lease_keepalive(self, lease: int) -> int:
        r = self._call("/v3/lease/keepalive", {"ID": str(lease)})
        return int((r.get("result") or {}).get("TTL", -1))

    def lease_revoke(self, lease: int):
        self._call("/v3/lease/revoke", {"ID": str(lease)})

    def keepalive_thread(self, lease: int, ttl: int,
                         on_lost: Optional[Callable[[], None]] = None) -> threading.Event:
        """Refresh ``lease`` every ttl/3 until the returned event is set.  If the
        server reports the lease gone (it expired while the KV was unreachable,
        or was revoked) the thread calls ``on_lost`` once and ends: the owner
        must grant a new lease and re-announce what hung off the old one."""
        stop = threading.Event()

        def run():
            while not stop.wait(max(0.5, ttl / 3)):
                try:
                    if self.lease_keepalive(lease) < 0:
                        if on_lost is not None and not stop.is_set():
                            on_lost()
                        return
                except KVError:
                    pass
        threading.Thread(target=run, daemon=True, name="pdo-kv-keepalive").start()
        return stop

    # -- watch --------------------------------------------------------------
    def watch(self, key: str, callback: Callable[[List[dict]], bool], prefix: bool = False,
              start_revision: int = 0, timeout: float = 3600.0):
        """Blocking watch; callback(events) → False stops. Events: {type, key, value, mod_revision}."""
        body = {"create_request": {"key": _b64(key)}}
        if prefix:
            body["create_request"]["range_end"] = _b64(prefix_end(key))
        if start_revision:
            body["create_request"]["start_revision"] = str(start_revision)
        host, port = self._host(self.endpoints[0])
        c = http.client.HTTPConnection(host, port, timeout=timeout)
        c.request("POST", "/v3/watch", json.dumps(body), {"Content-Type": "application/json"})
        r = c.getresponse()
        try:
            while True:
                line = r.readline()
                if not line:
                    return
                line = line.strip()
                if not line:
                    continue
                msg = json.loads(line).get("result", {})
                evs = []
                for e in msg.get("events") or []:
                    kv = e.get("kv", {})
                    evs.append({"type": e.get("type", "PUT"), "key": _unb64(kv.get("key")),
                                "value": _unb64(kv.get("value")), "mod_revision": int(kv.get("mod_revision", 0))})
                if evs and not callback(evs):
                    return
        finally:
            c.close()

    def wait_for(self, key: str, pred: Callable[[Optional[str]], bool], timeout: float = 60.0,
                 poll: float = 0.02) -> Optional[str]:
        t_end = time.time() + timeout
        while True:
            v = self.get(key)
            if pred(v):
                return v
            if time.time() > t_end:
                raise TimeoutError(f"kv wait_for {key} timed out")
            time.sleep(poll)

    def wait_count(self, prefix: str, n: int, timeout: float = 60.0, poll: float = 0.02) -> Dict[str, str]:
        t_end = time.time() + timeout
        while True:
            kv = self.get_prefix(prefix)
            if len(kv) >= n:
                return kv
            if time.time() > t_end:
                raise TimeoutError(f"kv wait_count {prefix} ({len(kv)}/{n}) timed out")
            time.sleep(poll)
