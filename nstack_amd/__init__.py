"""nstack_amd — MI355X-native Ethernet FCS engine (host-side mirror of nstack's FCS interface).

The product is the C-ABI library ``nstack_amd/libnstack_fcs.so`` (declared in
``include/nstack_fcs.h``): a gfx950 HIP kernel behind nstack's ``ether_fcs`` call surface
(/root/reference/src/ether_fcs.c:4, src/nstack_ether.h:80). This module is a thin ctypes
binding so Python tests, the bench and torch-based callers can drive it. It never computes a
CRC itself: if the library (or a GPU) is missing, every call raises ``FcsError``.
"""
from __future__ import annotations

import ctypes
import errno
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NSTACK_FCS_LIB") or os.path.join(_HERE, "libnstack_fcs.so")

__all__ = ["FcsError", "lib", "load", "ether_fcs", "fixed_dev", "batch_dev", "fixed_host",
           "batch_host", "tx_host", "tx_batch_host", "host_buffer", "host_free", "verify_dev", "verify_fixed_dev", "verify_host", "fill_splitmix_dev", "read_stream_dev", "timed_fixed_dev",
           "tables_blob", "TxQueue", "RxQueue", "set_var_threshold", "pcap_scan", "pcap_read", "pcap_write", "inet_batch_dev", "inet_fixed_dev", "inet_batch_host", "inet_set_flat_threshold", "inet_set_dma_threshold", "ip_checksum", "tcp_checksum", "udp_checksum", "INET_MODES", "engine_init", "engine_fini", "version", "LIB_PATH", "EXPORTS", "engine_stats", "shard_plan", "dma_stream_dev", "stream_load_dev", "load_faults", "FAULTS_PATH"]

# Every symbol include/nstack_fcs.h declares (tests check the .so exports all of them).
EXPORTS = [
    "ether_fcs", "fcs_engine_init", "fcs_engine_fini", "fcs_engine_device_count",
    "fcs_last_error", "fcs_engine_version", "fcs_engine_set_var_threshold", "fcs_engine_host_fallbacks", "fcs_engine_host_batches", "fcs_debug_stream_listed", "fcs_debug_stream_unit_frames", "fcs_debug_fixed_route", "fcs_debug_last_fixed_launch", "fcs_debug_device_syncs", "ether_fcs_batch_dev", "ether_fcs_fixed_dev",
    "ether_fcs_batch_host", "ether_fcs_fixed_host", "ether_fcs_tx_host", "ether_fcs_tx_batch_host", "ether_fcs_verify_dev",
    "ether_fcs_verify_fixed_dev", "ether_fcs_verify_host", "fcs_host_alloc",
    "fcs_host_free", "fcs_fill_splitmix64_dev", "fcs_read_stream_dev", "fcs_timed_fixed_dev",
    "fcs_tables_blob", "fcs_engine_stats", "fcs_engine_host_stats", "fcs_shard_plan", "fcs_dma_stream_dev", "fcs_stream_load_dev",
    "fcs_host_crc32",
    # include/nstack_txq.h — batched TX call site
    "fcs_txq_create", "fcs_txq_send", "fcs_txq_send_async", "fcs_txq_flush", "fcs_txq_destroy", "fcs_txq_stats", "fcs_txq_timing", "fcs_txq_last_error", "fcs_txq_fallbacks",
    "fcs_txq_set_host_max", "fcs_txq_set_sync_host", "fcs_txq_small_batches", "fcs_txq_sink_fd", "fcs_txq_sink_packet",
    # include/nstack_pcap.h — frame batches on disk
    "fcs_pcap_scan", "fcs_pcap_read", "fcs_pcap_write",
    # include/nstack_inet.h — batched Internet checksums (opt-in)
    "inet_csum_batch_dev", "inet_csum_fixed_dev", "inet_csum_batch_host", "inet_csum_set_flat_threshold", "inet_csum_set_dma_threshold", "inet_ip_checksum",
    "inet_tcp_checksum", "inet_udp_checksum",
    # include/nstack_rxq.h — batched RX call site with FCS verification
    "fcs_rxq_create", "fcs_rxq_receive", "fcs_rxq_stats", "fcs_rxq_fallbacks", "fcs_rxq_set_host_max",
    "fcs_rxq_small_batches", "fcs_rxq_destroy",
]

# include/nstack_inet.h modes: the reference function each result reproduces
INET_CSUM_IP, INET_CSUM_TCP, INET_CSUM_UDP = 0, 1, 2
INET_MODES = {"ip": INET_CSUM_IP, "tcp": INET_CSUM_TCP, "udp": INET_CSUM_UDP}


class FcsError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        name = errno.errorcode.get(-rc, str(rc)) if rc < 0 else str(rc)
        super().__init__(f"{what}: {name}: {_last_error()}")


_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the product library (raises FcsError with a clear message if it is not built)."""
    global _lib
    if _lib is not None:
        return _lib
    _lib = _bind(path)
    return _lib


FAULTS_PATH = os.path.join(_HERE, "libnstack_fcs_faults.so")
_faults = None


def load_faults() -> ctypes.CDLL:
    """The TEST-ONLY fault-hook build (-DFCS_FAULT_HOOK), bound like the product library plus its
    fcs_debug_fail_next / fcs_debug_timeout_next (drop-in) and fcs_debug_fail_batches /
    fcs_debug_late_batches (host batch calls: fail before the launch / give up after it with the
    kernel in flight) and fcs_debug_hold_small (the next small-batch launch waits behind a kernel
    that stays busy until a pinned host word turns nonzero) hooks. Its engine state is separate from the product library's. Nothing in the
    product loads it."""
    global _faults
    if _faults is None:
        L = _bind(FAULTS_PATH)
        for name in ("fcs_debug_fail_next", "fcs_debug_timeout_next"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [ctypes.c_int]
        for name in ("fcs_debug_fail_batches", "fcs_debug_late_batches"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [ctypes.c_int, ctypes.c_int]
        L.fcs_debug_retired.restype = ctypes.c_uint32
        L.fcs_debug_retired.argtypes = []
        L.fcs_debug_batch_faults_left.restype = ctypes.c_int
        L.fcs_debug_batch_faults_left.argtypes = []
        L.fcs_debug_hold_small.restype = None
        L.fcs_debug_hold_small.argtypes = [ctypes.c_void_p]
        _faults = L
    return _faults


def _bind(path: str) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise FcsError(-errno.ENOENT, f"{path} not built (run `make -C nstack_amd`)")
    L = ctypes.CDLL(path)
    c = ctypes
    u64, u32, vp, i32 = c.c_uint64, c.c_uint32, c.c_void_p, c.c_int
    sig = {
        "ether_fcs": (u32, [vp, c.c_size_t]),
        "fcs_engine_init": (i32, [i32]),
        "fcs_engine_fini": (None, []),
        "fcs_engine_device_count": (i32, []),
        "fcs_last_error": (c.c_char_p, []),
        "fcs_engine_version": (c.c_char_p, []),
        "fcs_engine_set_var_threshold": (u64, [u64]),
        "ether_fcs_batch_dev": (i32, [vp, u64, vp, vp, vp, u64, vp]),
        "ether_fcs_fixed_dev": (i32, [vp, u64, u32, u64, vp, vp]),
        "ether_fcs_batch_host": (i32, [vp, u64, vp, vp, vp, u64]),
        "ether_fcs_fixed_host": (i32, [vp, u64, u32, u64, vp]),
        "ether_fcs_tx_host": (i32, [vp, u64, vp, u64]),
        "ether_fcs_tx_batch_host": (i32, [vp, u64, vp, vp, u64]),
        "ether_fcs_verify_dev": (i32, [vp, u64, vp, vp, vp, vp, u64, vp]),
        "ether_fcs_verify_fixed_dev": (i32, [vp, u64, u32, u64, vp, vp, vp]),
        "ether_fcs_verify_host": (c.c_int64, [vp, u64, vp, vp, vp, u64]),
        "fcs_host_alloc": (vp, [u64]),
        "fcs_host_free": (None, [vp]),
        "fcs_fill_splitmix64_dev": (i32, [vp, u64, u64, u64, vp]),
        "fcs_read_stream_dev": (i32, [vp, u64, vp, vp]),
        "fcs_timed_fixed_dev": (i32, [vp, u64, u32, u64, vp, vp, i32, c.POINTER(c.c_float)]),
        "fcs_tables_blob": (i32, [vp, u64]),
        "fcs_engine_stats": (None, [c.POINTER(u64)] * 4),
        "fcs_engine_host_fallbacks": (u64, []),
        "fcs_engine_host_batches": (u64, []),
        "fcs_debug_stream_listed": (c.c_int64, []),
        "fcs_debug_stream_unit_frames": (u32, []),
        "fcs_debug_fixed_route": (i32, [u64, u64, u32, u64, c.c_char_p, u64]),
        "fcs_debug_last_fixed_launch": (i32, [c.c_char_p, u64]),
        "fcs_debug_device_syncs": (u64, []),
        "fcs_engine_host_stats": (None, [c.POINTER(u64)] * 2),
        "fcs_shard_plan": (i32, [vp, u64, u32, vp]),
        "fcs_dma_stream_dev": (i32, [vp, u64, vp, vp]),
        "fcs_stream_load_dev": (i32, [vp, u64, vp, vp, u64, vp, vp]),
        "fcs_txq_create": (vp, [vp, u32, u32, vp, vp]),
        "fcs_txq_send": (i32, [vp, vp, c.c_uint16, vp, c.c_size_t]),
        "fcs_txq_flush": (i32, [vp]),
        "fcs_txq_destroy": (None, [vp]),
        "fcs_txq_send_async": (i32, [vp, vp, c.c_uint16, vp, c.c_size_t]),
        "fcs_txq_stats": (None, [vp, c.POINTER(u64), c.POINTER(u64), c.POINTER(u64)]),
        "fcs_txq_timing": (None, [vp] + [c.POINTER(u64)] * 5),
        "fcs_txq_last_error": (c.c_char_p, [vp]),
        "fcs_txq_fallbacks": (None, [vp, c.POINTER(u64), c.POINTER(u64)]),
        "fcs_txq_set_host_max": (u64, [vp, u64]),
        "fcs_txq_set_sync_host": (i32, [vp, i32]),
        "fcs_txq_small_batches": (None, [vp, c.POINTER(u64), c.POINTER(u64), c.POINTER(u64)]),
        "fcs_host_crc32": (u32, [vp, c.c_size_t]),
        "fcs_txq_sink_fd": (None, [vp, vp, vp, vp, u32]),
        "fcs_txq_sink_packet": (None, [vp, vp, vp, vp, u32]),
        "fcs_pcap_scan": (i32, [c.c_char_p, c.POINTER(u64), c.POINTER(u64), c.POINTER(u32), c.POINTER(u64)]),
        "fcs_pcap_read": (c.c_int64, [c.c_char_p, vp, u64, vp, vp, u64]),
        "fcs_pcap_write": (i32, [c.c_char_p, vp, vp, vp, u64, u32]),
        "inet_csum_batch_dev": (i32, [i32, vp, u64, vp, vp, vp, vp, u64, vp]),
        "inet_csum_fixed_dev": (i32, [i32, vp, u64, u32, u64, vp, vp, vp]),
        "inet_csum_batch_host": (i32, [i32, vp, u64, vp, vp, vp, vp, u64]),
        "inet_csum_set_flat_threshold": (u64, [u64]),
        "inet_csum_set_dma_threshold": (u64, [u64]),
        "fcs_rxq_create": (vp, [i32, vp, u32, u32]),
        "fcs_rxq_receive": (i32, [vp, vp, vp, c.c_size_t]),
        "fcs_rxq_stats": (None, [vp] + [c.POINTER(u64)] * 5),
        "fcs_rxq_fallbacks": (None, [vp, c.POINTER(u64), c.POINTER(u64)]),
        "fcs_rxq_set_host_max": (u64, [vp, u64]),
        "fcs_rxq_small_batches": (None, [vp, c.POINTER(u64), c.POINTER(u64), c.POINTER(u64)]),
        "fcs_rxq_destroy": (None, [vp]),
        "inet_ip_checksum": (c.c_uint16, [vp, c.c_size_t]),
        "inet_tcp_checksum": (c.c_uint16, [u32, u32, vp, c.c_size_t]),
        "inet_udp_checksum": (c.c_uint16, [vp, c.c_size_t, u32, u32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def lib() -> ctypes.CDLL:
    return load()


def _last_error() -> str:
    if _lib is None:
        return ""
    s = _lib.fcs_last_error()
    return s.decode() if s else ""


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise FcsError(rc, what)
    return rc


def version() -> str:
    return load().fcs_engine_version().decode()


def engine_init(ndev: int = 0) -> int:
    return _check(load().fcs_engine_init(ndev), "fcs_engine_init")


def set_var_threshold(frames: int) -> int:
    """Variable-length batches of <= frames use the quarter-wave kernel; returns the old value."""
    return int(load().fcs_engine_set_var_threshold(frames))


def engine_fini() -> None:
    load().fcs_engine_fini()


def ether_fcs(data) -> int:
    """Drop-in single frame (src/ether_fcs.c:4): FCS of a bytes-like object, via the GPU."""
    b = bytes(data)
    return load().ether_fcs(b, len(b))


def _ptr(x):
    """Raw pointer of a torch tensor, numpy array, int, or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    raise TypeError(f"cannot take a pointer of {type(x)}")


def _stream(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)


def fixed_dev(base, stride: int, length: int, n: int, out, stream=None) -> None:
    _check(load().ether_fcs_fixed_dev(_ptr(base), stride, length, n, _ptr(out), _stream(stream)),
           "ether_fcs_fixed_dev")


def batch_dev(arena, arena_bytes: int, off, length, out, n: int, stream=None) -> None:
    _check(load().ether_fcs_batch_dev(_ptr(arena), arena_bytes, _ptr(off), _ptr(length), _ptr(out),
                                      n, _stream(stream)), "ether_fcs_batch_dev")


def fixed_host(base, stride: int, length: int, n: int, out) -> None:
    _check(load().ether_fcs_fixed_host(_ptr(base), stride, length, n, _ptr(out)),
           "ether_fcs_fixed_host")


def batch_host(arena, arena_bytes: int, off, length, out, n: int) -> None:
    _check(load().ether_fcs_batch_host(_ptr(arena), arena_bytes, _ptr(off), _ptr(length), _ptr(out),
                                       n), "ether_fcs_batch_host")


def tx_host(base, stride: int, length, n: int) -> None:
    _check(load().ether_fcs_tx_host(_ptr(base), stride, _ptr(length), n), "ether_fcs_tx_host")


def tx_batch_host(arena, arena_bytes: int, off, length, n: int) -> None:
    """TX mode over arena + offsets: the FCS of arena[off[i], +len[i]) lands at off[i] + len[i]."""
    _check(load().ether_fcs_tx_batch_host(_ptr(arena), arena_bytes, _ptr(off), _ptr(length), n),
           "ether_fcs_tx_batch_host")


def host_buffer(nbytes: int):
    """fcs_host_alloc'd (pinned, device-mapped) bytes as a numpy uint8 array; free with host_free."""
    import numpy as np
    p = load().fcs_host_alloc(nbytes)
    if not p:
        raise FcsError(f"fcs_host_alloc({nbytes}): {load().fcs_last_error().decode()}")
    return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))


def host_free(arr) -> None:
    load().fcs_host_free(arr.ctypes.data)


def verify_dev(arena, arena_bytes: int, off, length, ok, bad, n: int, stream=None) -> None:
    """RX check of frames that carry their FCS trailer: ok[i] (u8), *bad (u64) on the device."""
    _check(load().ether_fcs_verify_dev(_ptr(arena), arena_bytes, _ptr(off), _ptr(length), _ptr(ok),
                                       _ptr(bad), n, _stream(stream)), "ether_fcs_verify_dev")


def verify_fixed_dev(base, stride: int, length: int, n: int, ok, bad, stream=None) -> None:
    _check(load().ether_fcs_verify_fixed_dev(_ptr(base), stride, length, n, _ptr(ok), _ptr(bad),
                                             _stream(stream)), "ether_fcs_verify_fixed_dev")


def verify_host(arena, arena_bytes: int, off, length, ok, n: int) -> int:
    """Host form: fills ok[i] and returns the number of frames that fail the check."""
    return _check(load().ether_fcs_verify_host(_ptr(arena), arena_bytes, _ptr(off), _ptr(length),
                                               _ptr(ok), n), "ether_fcs_verify_host")


def fill_splitmix_dev(ptr, nbytes: int, seed: int, byte_offset: int = 0, stream=None) -> None:
    _check(load().fcs_fill_splitmix64_dev(_ptr(ptr), nbytes, seed, byte_offset, _stream(stream)),
           "fcs_fill_splitmix64_dev")


def dma_stream_dev(ptr, nbytes: int, sink, stream=None) -> None:
    _check(load().fcs_dma_stream_dev(_ptr(ptr), nbytes, _ptr(sink), _stream(stream)), "fcs_dma_stream_dev")


def stream_load_dev(arena, arena_bytes: int, off, length, n: int, sink, stream=None) -> None:
    """The arena-stream kernel's loads and schedule without its CRC work (fcs_stream_load_dev)."""
    _check(load().fcs_stream_load_dev(_ptr(arena), arena_bytes, _ptr(off), _ptr(length), n, _ptr(sink),
                                      _stream(stream)), "fcs_stream_load_dev")


def read_stream_dev(ptr, nbytes: int, sink, stream=None) -> None:
    _check(load().fcs_read_stream_dev(_ptr(ptr), nbytes, _ptr(sink), _stream(stream)),
           "fcs_read_stream_dev")


def timed_fixed_dev(base, stride: int, length: int, n: int, out, stream=None, reps: int = 10) -> float:
    ms = ctypes.c_float(0.0)
    _check(load().fcs_timed_fixed_dev(_ptr(base), stride, length, n, _ptr(out), _stream(stream),
                                      reps, ctypes.byref(ms)), "fcs_timed_fixed_dev")
    return float(ms.value)


def engine_stats() -> dict:
    """Drop-in ether_fcs health counters (fcs_engine_stats)."""
    import ctypes as c
    v = [c.c_uint64(0) for _ in range(4)]
    L = load()
    L.fcs_engine_stats(*[c.byref(x) for x in v])
    d = dict(zip(("dropin_calls", "dropin_retries", "dropin_recovered", "lane_resets"), (x.value for x in v)))
    d["host_fallbacks"] = int(L.fcs_engine_host_fallbacks())   # drop-in calls the host CRC answered
    d["host_batches"] = int(L.fcs_engine_host_batches())       # TX/RX queue batches the host CRC answered
    return d


def fixed_route(base: int, stride: int, length: int, n: int) -> str:
    """The kernel a fixed-length batch would take (fcs_debug_fixed_route; host arithmetic only)."""
    import ctypes
    buf = ctypes.create_string_buffer(64)
    _check(load().fcs_debug_fixed_route(base, stride, length, n, buf, 64), "fcs_debug_fixed_route")
    return buf.value.decode()


def last_fixed_launch() -> str:
    """"<route>/<threads>" of the kernel the last fixed-length launch actually launched."""
    import ctypes
    buf = ctypes.create_string_buffer(64)
    _check(load().fcs_debug_last_fixed_launch(buf, 64), "fcs_debug_last_fixed_launch")
    return buf.value.decode()


def stream_listed() -> int:
    """Units of the last arena-stream launch left to fcs_flat_kernel (fcs_debug_stream_listed)."""
    return int(load().fcs_debug_stream_listed())


def stream_unit_frames() -> int:
    """Frames per unit of the arena-stream kernel's dispenser (fcs_debug_stream_unit_frames)."""
    return int(load().fcs_debug_stream_unit_frames())


def engine_host_stats() -> dict:
    """Host batch calls split over several engine devices, and their shard jobs (fcs_engine_host_stats)."""
    import ctypes as c
    v = [c.c_uint64(0) for _ in range(2)]
    load().fcs_engine_host_stats(*[c.byref(x) for x in v])
    return {"sharded_calls": v[0].value, "shard_jobs": v[1].value}


def shard_plan(n: int, parts: int, lengths=None):
    """The engine's shard planner (fcs_shard_plan): cut points [0 .. n] of `parts` contiguous frame
    ranges, byte-balanced when `lengths` (uint32 per frame) is given. Host arithmetic only."""
    import numpy as np
    cut = np.zeros(parts + 1, dtype=np.uint64)
    ln = None if lengths is None else np.ascontiguousarray(lengths, dtype=np.uint32)
    _check(load().fcs_shard_plan(None if ln is None else ln.ctypes.data, n, parts, cut.ctypes.data),
           "fcs_shard_plan")
    return [int(x) for x in cut]


def tables_blob():
    import numpy as np
    buf = np.zeros(1 << 19, dtype=np.uint32)   # the blob is kBlobWords (about 261 k) words
    n = _check(load().fcs_tables_blob(buf.ctypes.data, buf.size), "fcs_tables_blob")
    return buf[:n].copy()


class TxQueue:
    """Batched ether_send (include/nstack_txq.h; src/linux/ether.c:214-272) over a connected
    socket fd: send() has ether_send's return contract (frame_size or -errno); frames from all
    threads are FCS'd together on the GPU and leave in one sendmmsg per batch."""

    def __init__(self, src_mac: bytes, fd: int, max_batch: int = 256, flush_usec: int = 0, sink=None,
                 sink_ctx=None, lib=None, host_max=None, gpu_only=False):
        """sink: None (fcs_txq_sink_fd on fd) or a C sink function pointer (e.g. fcs_txq_sink_packet)
        with sink_ctx its context pointer; lib: the library to use (default: the product); host_max:
        the GPU minimum of fire-and-forget batches in covered bytes (fcs_txq_set_host_max; None keeps
        the default); gpu_only: every frame, synchronous ones too, through a batch and its GPU step
        (host_max 0 and fcs_txq_set_sync_host off)."""
        L = self._L = lib or load()
        self._fd = ctypes.c_int(fd)
        self._mac = (ctypes.c_uint8 * 6)(*src_mac)
        if sink is None:
            sink, sink_ctx = ctypes.cast(L.fcs_txq_sink_fd, ctypes.c_void_p), ctypes.addressof(self._fd)
        self._q = L.fcs_txq_create(self._mac, max_batch, flush_usec, sink, sink_ctx)
        if not self._q:
            raise FcsError(-errno.EINVAL, "fcs_txq_create")
        if host_max is not None:
            L.fcs_txq_set_host_max(self._q, host_max)
        if gpu_only:
            L.fcs_txq_set_host_max(self._q, 0)
            L.fcs_txq_set_sync_host(self._q, 0)

    def send(self, dst: bytes, proto: int, payload: bytes) -> int:
        return self._L.fcs_txq_send(self._q, bytes(dst), proto, bytes(payload), len(payload))

    def send_async(self, dst: bytes, proto: int, payload: bytes) -> int:
        return self._L.fcs_txq_send_async(self._q, bytes(dst), proto, bytes(payload), len(payload))

    def flush(self) -> None:
        _check(self._L.fcs_txq_flush(self._q), "fcs_txq_flush")

    def stats(self):
        """(frames, batches, errors) since creation."""
        f, b, e = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._L.fcs_txq_stats(self._q, ctypes.byref(f), ctypes.byref(b), ctypes.byref(e))
        return int(f.value), int(b.value), int(e.value)

    def fallbacks(self):
        """(host_batches, host_frames): batches whose FCSs the host CRC computed (GPU step failed)."""
        hb, hf = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._L.fcs_txq_fallbacks(self._q, ctypes.byref(hb), ctypes.byref(hf))
        return int(hb.value), int(hf.value)

    def set_host_max(self, nbytes: int) -> int:
        """Set the GPU minimum (covered bytes); returns the previous value."""
        return int(self._L.fcs_txq_set_host_max(self._q, nbytes))

    def paths(self):
        """(small_batches, small_frames, gpu_batches): batches at or below the GPU minimum (host CRC by
        design) and batches the GPU computed."""
        sb, sf, gb = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._L.fcs_txq_small_batches(self._q, ctypes.byref(sb), ctypes.byref(sf), ctypes.byref(gb))
        return int(sb.value), int(sf.value), int(gb.value)

    def last_error(self) -> str:
        """Text of the most recent failed GPU step ("" if none)."""
        return (self._L.fcs_txq_last_error(self._q) or b"").decode()

    def close(self) -> None:
        if self._q:
            self._L.fcs_txq_destroy(self._q)
            self._q = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class RxQueue:
    """Batched ether_receive (include/nstack_rxq.h; src/linux/ether.c:180-212) on a socket fd:
    receive() returns (payload_len, dst, src, proto, payload) like ether_receive (0 = nothing
    queued, negative = -errno); with trailer=True every recvmmsg batch is FCS-verified on the GPU,
    failing frames are dropped and the 4-byte trailer is stripped."""

    def __init__(self, fd: int, own_mac: bytes, max_batch: int = 64, trailer: bool = True, lib=None,
                 host_max=None):
        """host_max: the GPU minimum in bytes (fcs_rxq_set_host_max; None keeps the default, 0 checks
        every batch on the GPU)."""
        L = self._L = lib or load()
        self._mac = (ctypes.c_uint8 * 6)(*own_mac)
        self._q = L.fcs_rxq_create(fd, self._mac, max_batch, 1 if trailer else 0)
        if not self._q:
            raise FcsError(-errno.EINVAL, "fcs_rxq_create")
        if host_max is not None:
            L.fcs_rxq_set_host_max(self._q, host_max)
        self._hdr = (ctypes.c_uint8 * 14)()
        self._buf = (ctypes.c_uint8 * 2048)()

    def receive(self, bsize: int = 2048):
        r = self._L.fcs_rxq_receive(self._q, self._hdr, self._buf, min(bsize, 2048))
        if r <= 0:
            return r, None, None, None, b""
        h = bytes(self._hdr)
        proto = int.from_bytes(h[12:14], "little")   # host-order u16 in the struct
        return r, h[0:6], h[6:12], proto, bytes(self._buf[:min(r, bsize)])

    def stats(self):
        """(frames, bad_fcs, echoes, dropped, batches) since creation."""
        v = [ctypes.c_uint64(0) for _ in range(5)]
        self._L.fcs_rxq_stats(self._q, *[ctypes.byref(x) for x in v])
        return tuple(int(x.value) for x in v)

    def fallbacks(self):
        """(host_batches, host_frames): batches the host CRC checked because the GPU check failed."""
        hb, hf = ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._L.fcs_rxq_fallbacks(self._q, ctypes.byref(hb), ctypes.byref(hf))
        return int(hb.value), int(hf.value)

    def paths(self):
        """(small_batches, small_frames, gpu_batches): batches the host CRC checked by design (at or
        below the GPU minimum) and batches the GPU checked."""
        sb, sf, gb = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._L.fcs_rxq_small_batches(self._q, ctypes.byref(sb), ctypes.byref(sf), ctypes.byref(gb))
        return int(sb.value), int(sf.value), int(gb.value)

    def close(self) -> None:
        if self._q:
            self._L.fcs_rxq_destroy(self._q)
            self._q = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def pcap_scan(path: str):
    """(frames, captured bytes, link type, truncated records) of a classic pcap file."""
    n, b, t = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    lt = ctypes.c_uint32(0)
    _check(load().fcs_pcap_scan(os.fsencode(path), ctypes.byref(n), ctypes.byref(b), ctypes.byref(lt),
                                ctypes.byref(t)), "fcs_pcap_scan")
    return int(n.value), int(b.value), int(lt.value), int(t.value)


def pcap_read(path: str):
    """Load a pcap into the batch layout: (arena u8, off u64, len u32, link type) as numpy arrays."""
    import numpy as np
    n, b, lt, _ = pcap_scan(path)
    arena = np.empty(max(b, 1), dtype=np.uint8)   # every byte of [0, b) is written by the read
    off = np.zeros(max(n, 1), dtype=np.uint64)
    ln = np.zeros(max(n, 1), dtype=np.uint32)
    got = _check(load().fcs_pcap_read(os.fsencode(path), arena.ctypes.data, arena.size, off.ctypes.data,
                                      ln.ctypes.data, n), "fcs_pcap_read")
    return arena[:b], off[:got], ln[:got], lt


def pcap_write(path: str, arena, off, length, linktype: int = 1) -> None:
    import numpy as np
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    _check(load().fcs_pcap_write(os.fsencode(path), _ptr(arena), off.ctypes.data, length.ctypes.data,
                                 len(off), linktype), "fcs_pcap_write")


# ---- Internet checksums (include/nstack_inet.h; src/ip.c:39, src/tcp.c:167, src/udp.c:136) ----
def _mode(mode) -> int:
    return INET_MODES[mode] if isinstance(mode, str) else int(mode)


def inet_batch_dev(mode, arena, arena_bytes: int, off, length, addr, out, n: int, stream=None) -> None:
    """out[i] (u16) = the reference checksum of arena[off[i]:off[i]+len[i]] (device arrays)."""
    _check(load().inet_csum_batch_dev(_mode(mode), _ptr(arena), arena_bytes, _ptr(off), _ptr(length),
                                      _ptr(addr), _ptr(out), n, _stream(stream)), "inet_csum_batch_dev")


def inet_fixed_dev(mode, base, stride: int, length: int, n: int, addr, out, stream=None) -> None:
    _check(load().inet_csum_fixed_dev(_mode(mode), _ptr(base), stride, length, n, _ptr(addr), _ptr(out),
                                      _stream(stream)), "inet_csum_fixed_dev")


def inet_batch_host(mode, arena, arena_bytes: int, off, length, addr, out, n: int) -> None:
    _check(load().inet_csum_batch_host(_mode(mode), _ptr(arena), arena_bytes, _ptr(off), _ptr(length),
                                       _ptr(addr), _ptr(out), n), "inet_csum_batch_host")


def inet_set_flat_threshold(packets: int) -> int:
    """Variable-length batches of more than `packets` packets use the flat kernel; returns the old value."""
    return int(load().inet_csum_set_flat_threshold(packets))


def inet_set_dma_threshold(packets: int) -> int:
    """Fixed-stride batches of more than `packets` packets use the LDS-DMA kernel (when their
    geometry fits its slots); returns the old value."""
    return int(load().inet_csum_set_dma_threshold(packets))


def ip_checksum(data) -> int:
    """ip_checksum(dp, bsize) of src/ip.c:39-62, computed on the GPU."""
    b = bytes(data)
    return load().inet_ip_checksum(b, len(b))


def tcp_checksum(src: int, dst: int, data) -> int:
    """tcp_checksum(&src, &dst, dp, bsize) of src/tcp.c:167-213 (host-order addresses)."""
    b = bytes(data)
    return load().inet_tcp_checksum(src, dst, b, len(b))


def udp_checksum(data, src: int, dst: int) -> int:
    """udp_checksum(buff, len, src, dst) of src/udp.c:136-174 (raw in_addr_t values)."""
    b = bytes(data)
    return load().inet_udp_checksum(b, len(b), src, dst)
