"""Loader for the in-tree native extensions.

Two shared objects live next to this file once ``tools/build.py`` has run:

* ``_pdo_hip.so``  — hand-written HIP/CDNA4 kernels (``csrc/hip``) bound to
  PyTorch tensors through pybind11 (hipcc-compiled for gfx950, no hipify).
* ``_pdo_core.so`` — the native control plane (``csrc/core``): JSON DOM,
  PaddleJob builders, phase FSM, planner, host-port allocator.

Policy (MI355X-first): on a machine with a visible GPU the HIP extension is
REQUIRED — a missing or stale build raises instead of silently running the
PyTorch reference path.  ``PDO_OPS=torch`` is an explicit, logged opt-out used
only for A/B measurements against the reference implementation.
"""
from __future__ import annotations

import importlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))

_hip = None
_hip_err: Exception | None = None
_core = None
_core_err: Exception | None = None


def _load(name: str):
    if _HERE not in sys.path:
        pass
    return importlib.import_module(f"paddle_operator_amd.{name}")


def hip_ext():
    """Return the HIP kernel module or ``None`` (CPU-only container)."""
    global _hip, _hip_err
    if _hip is not None or _hip_err is not None:
        return _hip
    try:
        import torch  # noqa: F401  (libtorch must be loaded first)
        _hip = _load("_pdo_hip")
    except Exception as e:  # pragma: no cover - depends on build state
        _hip_err = e
    return _hip


def hip_error():
    return _hip_err


def ops_mode() -> str:
    """``hip`` (default) or ``torch`` (reference path, explicit opt-out)."""
    return os.environ.get("PDO_OPS", "hip").lower()


def require_hip():
    """The HIP module, or raise loudly: used on every GPU code path."""
    m = hip_ext()
    if m is None:
        raise RuntimeError(
            "paddle_operator_amd: HIP extension _pdo_hip is not built/loadable "
            f"({_hip_err!r}). Run `python tools/build.py` (hipcc --offload-arch=gfx950).")
    return m


def core_ext():
    global _core, _core_err
    if _core is not None or _core_err is not None:
        return _core
    try:
        _core = _load("_pdo_core")
    except Exception as e:  # pragma: no cover
        _core_err = e
    return _core


def require_core():
    m = core_ext()
    if m is None:
        raise RuntimeError(
            "paddle_operator_amd: native control-plane module _pdo_core is not built "
            f"({_core_err!r}). Run `python tools/build.py`.")
    return m
