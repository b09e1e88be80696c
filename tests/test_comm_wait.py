"""The bounded host wait of a rank whose step carries RCCL all-reduces (csrc/comm_wait.h), driven through the C ABI's
test hook with mocked probes — no device needed. The all-reduce points it guards replace the reference's local
wo / down outputs (source/model/model.cpp:86-90, 124-128); the wait itself is the reference's per-token sync at the
logits copy (model.cpp:175-179). A wedged communicator must end the wait with an error code, never hang it."""
import ctypes
import time

from simplellminference_amd import _lib


def _wait(mode, deadline_ms):
    waited = ctypes.c_double()
    rc = _lib.load().sli_debug_bounded_wait(mode, deadline_ms, ctypes.byref(waited))
    return rc, waited.value, _lib.load().sli_last_error().decode()


def test_completing_query_returns_ok():
    rc, waited, _ = _wait(0, 5000.0)
    assert rc == _lib.SLI_OK and waited < 1000.0


def test_never_completing_query_times_out_at_the_deadline():
    t0 = time.perf_counter()
    rc, waited, msg = _wait(1, 300.0)
    wall = (time.perf_counter() - t0) * 1e3
    assert rc == _lib.SLI_ERR_TIMEOUT, (rc, msg)
    assert 300.0 <= waited <= 1500.0 and wall < 3000.0
    assert "wedged" in msg and "SLI_COMM_TIMEOUT_MS" in msg


def test_async_communicator_error_ends_the_wait():
    rc, waited, msg = _wait(2, 60000.0)
    assert rc == _lib.SLI_ERR_COMM and waited < 1000.0
    assert "mocked remote error" in msg


def test_failed_query_is_a_hip_error():
    rc, _, _ = _wait(3, 60000.0)
    assert rc == 4  # SLI_ERR_HIP


def test_status_string():
    assert _lib.load().sli_status_str(_lib.SLI_ERR_TIMEOUT).decode() == "communicator wait timed out"


def test_bad_arguments_rejected():
    waited = ctypes.c_double()
    assert _lib.load().sli_debug_bounded_wait(7, 1.0, ctypes.byref(waited)) == 1


def test_bench_exits_nonzero_on_a_wedged_rank():
    """bench.py turns these codes into a non-zero exit of the rank (no retry, no re-exec): _comm_fatal."""
    import bench
    assert bench._comm_fatal(_lib.SliError(_lib.SLI_ERR_TIMEOUT, "sli_model_sync", "x")) is True
    assert bench._comm_fatal(_lib.SliError(_lib.SLI_ERR_COMM, "sli_model_sync", "x")) is True
    assert bench._comm_fatal(_lib.SliError(2, "sli_model_step", "x")) is False
    assert bench._comm_fatal(ValueError("x")) is False
