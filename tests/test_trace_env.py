"""roctx tracing helper (utils/trace.py) and the context-parallel extension point."""
import pytest

from paddle_operator_amd.utils import trace


def test_trace_disabled_is_noop():
    trace.enable(False)
    with trace.range("x") as r:
        assert r is None
    trace.mark("m")


def test_trace_enabled_pushes_and_pops():
    if not trace.enable(True):
        pytest.skip("libroctx64 not present")
    try:
        with trace.range("outer"):
            with trace.range("inner"):
                trace.mark("here")
    finally:
        trace.enable(False)


def test_cp_size_extension_point_fails_loudly():
    from paddle_operator_amd.launch.env import JobEnv

    JobEnv.from_env({"PADDLE_TRAINER_ID": "0"}).check_supported()
    with pytest.raises(NotImplementedError):
        JobEnv.from_env({"PDO_CP_SIZE": "2"}).check_supported()
