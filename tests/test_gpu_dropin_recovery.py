"""The drop-in's error contract (SURVEY.md §8b Errors; /root/reference/src/ether_fcs.c:4-19 cannot
fail): a failed attempt is retried once on a fresh lane; if the retry fails too, the library's own
host CRC answers (counted in fcs_engine_host_fallbacks). The caller always gets the right FCS.

Runs against nstack_amd/libnstack_fcs_faults.so, the test-only build with -DFCS_FAULT_HOOK:
fcs_debug_fail_next(k) makes the calling thread's next k drop-in attempts fail as if the GPU step
had returned an error, and fcs_debug_timeout_next(k) makes the next k single-frame attempts give up
right after their launch as if the 10 s wait had run out, with the kernel still in flight (the
lane's stream and result word are quarantined, as on a real failure). The product library has no
such hooks."""
import ctypes
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAULTS = os.path.join(ROOT, "nstack_amd", "libnstack_fcs_faults.so")


@pytest.fixture(scope="module")
def flib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(FAULTS):
        pytest.fail("libnstack_fcs_faults.so not built (make -C nstack_amd)")
    L = ctypes.CDLL(FAULTS)
    L.ether_fcs.restype = ctypes.c_uint32
    L.ether_fcs.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.fcs_debug_fail_next.argtypes = [ctypes.c_int]
    L.fcs_debug_timeout_next.argtypes = [ctypes.c_int]
    L.fcs_engine_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)] * 4
    L.fcs_engine_host_fallbacks.restype = ctypes.c_uint64
    return L


def stats(L):
    v = [ctypes.c_uint64(0) for _ in range(4)]
    L.fcs_engine_stats(*[ctypes.byref(x) for x in v])
    return [x.value for x in v]


def fcs(L, b: bytes):
    buf = ctypes.create_string_buffer(b, len(b))
    return L.ether_fcs(buf, len(b))


@pytest.mark.parametrize("L", [9, 64, 1514, 1536, 1537, 4000, 9000])
def test_forced_first_attempt_failure_still_returns_the_fcs(flib, L):
    rng = np.random.default_rng(L)
    frame = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
    assert fcs(flib, frame) == zlib.crc32(frame)            # healthy lanes first
    c0, r0, ok0, z0 = stats(flib)
    flib.fcs_debug_fail_next(1)
    assert fcs(flib, frame) == zlib.crc32(frame)
    c1, r1, ok1, z1 = stats(flib)
    assert (c1 - c0, r1 - r0, ok1 - ok0) == (1, 1, 1)
    assert z1 - z0 >= 1                                       # the failed lane was dropped
    for _ in range(3):                                        # and later calls run normally
        assert fcs(flib, frame) == zlib.crc32(frame)
    assert stats(flib)[1] == r1


def test_recovery_under_concurrent_callers(flib):
    import threading
    rng = np.random.default_rng(5)
    frames = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(1, 1536, 64)]
    errors = []

    def worker(k):
        for i, f in enumerate(frames[k::4]):
            if i % 5 == 0:
                flib.fcs_debug_fail_next(1)
            if fcs(flib, f) != zlib.crc32(f):
                errors.append((k, i))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors


@pytest.mark.parametrize("L", [9, 1514, 1536, 4000])
def test_both_attempts_fail_host_crc_answers(flib, L):
    """First attempt and retry both fail: the host CRC answers, counted, no abort."""
    rng = np.random.default_rng(L + 11)
    frame = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
    h0 = flib.fcs_engine_host_fallbacks()
    c0, r0, ok0, _ = stats(flib)
    flib.fcs_debug_fail_next(2)
    assert fcs(flib, frame) == zlib.crc32(frame)
    c1, r1, ok1, _ = stats(flib)
    assert flib.fcs_engine_host_fallbacks() == h0 + 1
    assert (c1 - c0, r1 - r0, ok1 - ok0) == (1, 1, 0)
    h1 = flib.fcs_engine_host_fallbacks()
    for _ in range(3):                                        # the GPU path serves the next calls
        assert fcs(flib, frame) == zlib.crc32(frame)
    assert flib.fcs_engine_host_fallbacks() == h1


def test_timeout_with_kernel_in_flight_quarantines_the_lane(flib):
    """a lane given up while its kernel may still run is quarantined, not freed. The
    injected timeout leaves the launched kernel in flight; the retry runs on a fresh lane; a second
    injected timeout sends the call to the host CRC; later calls reuse no quarantined word."""
    rng = np.random.default_rng(21)
    frames = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in (60, 1514, 777)]
    c0, r0, ok0, z0 = stats(flib)
    h0 = flib.fcs_engine_host_fallbacks()
    flib.fcs_debug_timeout_next(1)
    assert fcs(flib, frames[0]) == zlib.crc32(frames[0])
    c1, r1, ok1, z1 = stats(flib)
    assert (r1 - r0, ok1 - ok0) == (1, 1) and z1 - z0 == 1
    flib.fcs_debug_timeout_next(2)
    assert fcs(flib, frames[1]) == zlib.crc32(frames[1])
    assert flib.fcs_engine_host_fallbacks() == h0 + 1
    for _ in range(50):   # the quarantined words may still be written by the late kernels
        for f in frames:
            assert fcs(flib, f) == zlib.crc32(f)
    assert flib.fcs_engine_host_fallbacks() == h0 + 1
