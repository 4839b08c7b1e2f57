"""the host batch forms answer a failed GPU step from the product's host
CRC, so their results never differ from the reference's.

The reference's ether_fcs (/root/reference/src/ether_fcs.c:4-19) cannot fail. Its batch forms here
(ether_fcs_batch_host, ether_fcs_fixed_host, ether_fcs_tx_host, ether_fcs_tx_batch_host,
ether_fcs_verify_host; include/nstack_fcs.h) keep -EINVAL for bad arguments and -ENODEV when no
gfx950 GPU or code object is usable at all; any other failure of their GPU step is answered by
nstack_amd/csrc/fcs_host_crc.cpp (the product's slice-by-16, not the oracle), counted in
fcs_engine_host_batches, reported once on stderr.

Runs against nstack_amd/libnstack_fcs_faults.so (-DFCS_FAULT_HOOK):
  fcs_debug_fail_batches(skip, calls)  the call fails at entry, before anything is launched;
  fcs_debug_late_batches(skip, calls)  the call gives up at its first wait after the launch, with
                                       the kernel still in flight, as a timeout would.
Every path each form takes is driven through both: the staged pipeline (pageable memory), the
zero-copy kernels on fcs_host_alloc memory (small list in the kernel arguments, and the arena
kernels for larger batches), and the one-frame kernel. Expected values come from the oracle; every
check is exact. The suite's last file asserts the PRODUCT library's fcs_engine_host_batches is 0.
"""
import ctypes

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

RESIDUE = 0x2144DF1C


@pytest.fixture(scope="module")
def flib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = na.load_faults()
    yield L
    L.fcs_debug_fail_batches(0, 0)
    L.fcs_debug_late_batches(0, 0)


def _arm(flib, mode):
    (flib.fcs_debug_fail_batches if mode == "entry" else flib.fcs_debug_late_batches)(0, 1)


def _frames(n, seed, fixed=None, tail=0):
    """Packed frames (lengths 0..1600, or `fixed`), each followed by `tail` spare bytes."""
    rng = np.random.default_rng(seed)
    ln = np.full(n, fixed, dtype=np.uint32) if fixed is not None else rng.integers(0, 1601, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + tail)
    size = int(off[-1]) + int(ln[-1]) + tail
    return ln, off, size, rng


def _fill(buf, rng):
    buf[:] = rng.integers(0, 256, buf.size, dtype=np.uint8)


def _oracle_var(oracle, arena, off, ln):
    out = np.zeros(len(ln), dtype=np.uint32)
    oracle.oracle_fcs_batch(arena.ctypes.data, off.ctypes.data, ln.ctypes.data, out.ctypes.data, len(ln), 1)
    return out


class _Host:
    """Pageable numpy memory, or fcs_host_alloc memory of the faults library (the zero-copy paths)."""

    def __init__(self, flib, pinned):
        self.flib, self.pinned, self.keep = flib, pinned, []

    def bytes(self, n):
        if not self.pinned:
            return np.zeros(max(n, 1), dtype=np.uint8)
        p = self.flib.fcs_host_alloc(max(n, 1))
        assert p
        self.keep.append(p)
        return np.ctypeslib.as_array((ctypes.c_uint8 * max(n, 1)).from_address(p))

    def array(self, a):
        b = self.bytes(a.nbytes).view(a.dtype)[:a.size]
        b[:] = a
        return b

    def free(self):
        torch.cuda.synchronize()   # a kernel given up on by a late fault may still read this memory
        for p in self.keep:
            self.flib.fcs_host_free(p)


CASES = [(1, False), (40, False), (3000, False), (1, True), (40, True), (3000, True)]


def _call(flib, form, oracle, n, pinned, seed):
    """Run one host form on fresh frames; returns (return value, results exact)."""
    h = _Host(flib, pinned)
    try:
        if form == "fixed":
            L = 1518
            arena = h.bytes(n * L)
            _fill(arena, np.random.default_rng(seed))
            out = np.zeros(n, dtype=np.uint32)
            rc = flib.ether_fcs_fixed_host(arena.ctypes.data, L, L, n, out.ctypes.data)
            exp = np.zeros(n, dtype=np.uint32)
            oracle.oracle_fcs_fixed(arena.ctypes.data, L, L, n, exp.ctypes.data, 1, 1)
            return rc, np.array_equal(out, exp)
        if form == "batch":
            ln, off, size, rng = _frames(n, seed)
            arena = h.bytes(size)
            _fill(arena, rng)
            out = np.zeros(n, dtype=np.uint32)
            rc = flib.ether_fcs_batch_host(arena.ctypes.data, size, off.ctypes.data, ln.ctypes.data, out.ctypes.data, n)
            return rc, np.array_equal(out, _oracle_var(oracle, arena, off, ln))
        if form == "tx":
            stride = 1536
            ln = np.random.default_rng(seed).integers(0, stride - 3, n).astype(np.uint32)
            base = h.bytes(n * stride)
            _fill(base, np.random.default_rng(seed + 1))
            off = (np.arange(n, dtype=np.uint64) * stride)
            want = _oracle_var(oracle, base, off, ln)
            rc = flib.ether_fcs_tx_host(base.ctypes.data, stride, ln.ctypes.data, n)
            got = np.array([int.from_bytes(bytes(base[int(o) + int(l):int(o) + int(l) + 4]), "little")
                            for o, l in zip(off, ln)], dtype=np.uint32)
            return rc, np.array_equal(got, want)
        if form == "tx_batch":
            ln, off, size, rng = _frames(n, seed, tail=4)
            ln = np.minimum(ln, 1536).astype(np.uint32)
            off = h.array(off)
            ln = h.array(ln)
            arena = h.bytes(size)
            _fill(arena, rng)
            want = _oracle_var(oracle, arena, off, ln)
            rc = flib.ether_fcs_tx_batch_host(arena.ctypes.data, size, off.ctypes.data, ln.ctypes.data, n)
            got = np.array([int.from_bytes(bytes(arena[int(o) + int(l):int(o) + int(l) + 4]), "little")
                            for o, l in zip(off, ln)], dtype=np.uint32)
            return rc, np.array_equal(got, want)
        # verify: frames carrying their FCS trailer, every third one corrupted
        ln, off, size, rng = _frames(n, seed)
        ln = np.maximum(ln, 4).astype(np.uint32)
        off = np.zeros(n, dtype=np.uint64)
        if n > 1:
            off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
        size = int(off[-1]) + int(ln[-1])
        arena = h.bytes(size)
        _fill(arena, rng)
        for i in range(n):
            o, L = int(off[i]), int(ln[i])
            c = oracle.oracle_crc32_fast(arena[o:].ctypes.data, L - 4)
            arena[o + L - 4:o + L] = np.frombuffer(int(c).to_bytes(4, "little"), dtype=np.uint8)
            if i % 3 == 2:
                arena[o + int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))
        off, ln = h.array(off), h.array(ln)
        ok = h.bytes(n)
        want = (_oracle_var(oracle, arena, off, ln) == RESIDUE).astype(np.uint8)
        rc = flib.ether_fcs_verify_host(arena.ctypes.data, size, off.ctypes.data, ln.ctypes.data, ok.ctypes.data, n)
        return rc, np.array_equal(ok[:n], want) and rc == int(n - want.sum())
    finally:
        h.free()


@pytest.mark.parametrize("form", ["batch", "fixed", "tx", "tx_batch", "verify"])
@pytest.mark.parametrize("mode", ["entry", "late"])
@pytest.mark.parametrize("n,pinned", CASES)
def test_host_form_failure_answered_by_host_crc(flib, oracle, form, mode, n, pinned):
    """One failed call of each host form on each of its paths: the results are exact, the call
    succeeds, exactly one call is counted, and a failure after the launch retires what the kernel
    in flight can still write (the one-frame TX kernel: its lane)."""
    flib.fcs_engine_fini()   # a fresh engine: earlier cases' retirements must not reach host-only mode
    flib.fcs_engine_init(0)
    h0, r0 = flib.fcs_engine_host_batches(), flib.fcs_debug_retired()
    lanes0 = ctypes.c_uint64(0)
    flib.fcs_engine_stats(None, None, None, ctypes.byref(lanes0))
    _arm(flib, mode)
    rc, exact = _call(flib, form, oracle, n, pinned, 1000 * n + len(form))
    assert flib.fcs_debug_batch_faults_left() == 0
    assert rc >= 0 and exact
    assert flib.fcs_engine_host_batches() - h0 == 1
    err = flib.fcs_last_error().decode()
    assert "answered by the host CRC" in err and "injected" in err
    lanes = ctypes.c_uint64(0)
    flib.fcs_engine_stats(None, None, None, ctypes.byref(lanes))
    if mode == "late":
        one_frame_tx = n == 1 and form in ("tx", "tx_batch")
        assert (lanes.value - lanes0.value == 1) if one_frame_tx else (flib.fcs_debug_retired() - r0 == 1)
    else:
        assert flib.fcs_debug_retired() == r0
    # the next call runs on the GPU again (fresh staging / stream), exact and not counted
    rc, exact = _call(flib, form, oracle, n, pinned, 1000 * n + len(form) + 7)
    assert rc >= 0 and exact
    assert flib.fcs_engine_host_batches() - h0 == 1


def test_bad_arguments_stay_einval(flib):
    """-EINVAL is never answered by the host CRC: nothing is written, nothing is counted."""
    h0 = flib.fcs_engine_host_batches()
    arena = np.zeros(100, dtype=np.uint8)
    off = np.array([90], dtype=np.uint64)
    ln = np.array([20], dtype=np.uint32)
    out = np.full(1, 7, dtype=np.uint32)
    assert flib.ether_fcs_batch_host(arena.ctypes.data, 100, off.ctypes.data, ln.ctypes.data, out.ctypes.data, 1) == -22
    assert out[0] == 7
    assert flib.ether_fcs_tx_host(arena.ctypes.data, 10, ln.ctypes.data, 1) == -22
    assert flib.fcs_engine_host_batches() == h0


def test_late_tx_kernel_never_writes_the_reused_arena(flib, oracle):
    """A zero-copy TX call gives up with its kernel in flight; the caller at once refills the same
    pinned arena with other frames and sends them: the FCSs in the arena are exactly the second
    batch's (the late kernel writes the engine's retired result array, never the frames)."""
    n, stride = 48, 1536
    p = flib.fcs_host_alloc(n * stride)
    try:
        base = np.ctypeslib.as_array((ctypes.c_uint8 * (n * stride)).from_address(p))
        off = np.arange(n, dtype=np.uint64) * stride
        for rnd in range(6):
            rng = np.random.default_rng(rnd)
            ln = rng.integers(60, 1515, n).astype(np.uint32)
            base[:] = rng.integers(0, 256, base.size, dtype=np.uint8)
            if rnd % 2 == 0:
                flib.fcs_debug_late_batches(0, 1)
            assert flib.ether_fcs_tx_host(p, stride, ln.ctypes.data, n) == 0
            want = _oracle_var(oracle, base, off, ln)
            got = np.array([int.from_bytes(bytes(base[int(o) + int(l):int(o) + int(l) + 4]), "little")
                            for o, l in zip(off, ln)], dtype=np.uint32)
            assert np.array_equal(got, want), rnd
    finally:
        torch.cuda.synchronize()
        flib.fcs_host_free(p)


def test_host_only_after_repeated_late_failures(flib, oracle):
    """After 16 retirements the host forms answer from the host CRC without calling the GPU (the
    remaining armed faults are not consumed); fcs_engine_fini frees the retired resources and the
    next call runs on the GPU again."""
    flib.fcs_engine_fini()
    flib.fcs_engine_init(0)
    assert flib.fcs_debug_retired() == 0
    h0 = flib.fcs_engine_host_batches()
    flib.fcs_debug_late_batches(0, 20)
    for i in range(20):
        rc, exact = _call(flib, "tx_batch", oracle, 40, True, 50 + i)
        assert rc == 0 and exact, i
    assert flib.fcs_debug_retired() == 16
    assert flib.fcs_debug_batch_faults_left() == 4     # calls 17..20 made no GPU call at all
    assert flib.fcs_engine_host_batches() - h0 == 20
    assert "stopped using the GPU" in flib.fcs_last_error().decode()
    flib.fcs_debug_late_batches(0, 0)
    flib.fcs_engine_fini()
    assert flib.fcs_debug_retired() == 0
    rc, exact = _call(flib, "tx_batch", oracle, 40, True, 99)
    assert rc == 0 and exact
    assert flib.fcs_engine_host_batches() - h0 == 20
