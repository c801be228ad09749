"""roctx ranges for rocprofv3 timelines ("add roctx ranges in the
launcher").

The reference has no tracing at all (only k8s Events and
status.startTime/completionTime, controllers/paddlejob_helper.go:175-189).
Here the launcher and the GPT-2 trainer mark their phases (step, forward,
backward, all-reduce drain, optimizer, checkpoint) so a
``rocprofv3 --marker-trace --kernel-trace`` timeline groups kernels by phase.

Calls go straight to rocprofiler-sdk's roctx library through ctypes (no torch wrapper).
Disabled unless ``PDO_ROCTX=1``: then ``range()`` is a shared no-op context
manager, so the instrumented hot loop pays one attribute lookup per phase.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_LIB = None
_ENABLED = os.environ.get("PDO_ROCTX", "0") == "1"
_NULL = contextlib.nullcontext()


def _lib():
    global _LIB, _ENABLED
    if _LIB is None:
        lib_dir = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")
        # rocprofiler-sdk's roctx first: rocprofv3 --marker-trace intercepts it
        # (the legacy roctracer libroctx64 is not seen by rocprofv3)
        for name in (os.path.join(lib_dir, "librocprofiler-sdk-roctx.so.1"),
                     os.path.join(lib_dir, "libroctx64.so.4"), "libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
            except OSError:
                continue
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.restype = None
            _LIB = lib
            break
        else:
            _ENABLED = False  # no roctx on this host: stay a no-op
    return _LIB


def enabled() -> bool:
    return _ENABLED and _lib() is not None


def enable(on: bool = True) -> bool:
    """Turn ranges on/off at run time; returns whether roctx is active."""
    global _ENABLED
    _ENABLED = bool(on)
    return enabled()


class _Range:
    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = name.encode()

    def __enter__(self):
        _LIB.roctxRangePushA(self.name)
        return self

    def __exit__(self, *exc):
        _LIB.roctxRangePop()
        return False


def range(name: str):  # noqa: A001 - mirrors roctx naming
    """``with trace.range("backward"): ...`` — a roctx push/pop pair when enabled."""
    if not _ENABLED or _lib() is None:
        return _NULL
    return _Range(name)


def mark(name: str) -> None:
    if _ENABLED and _lib() is not None:
        _LIB.roctxMarkA(name.encode())
