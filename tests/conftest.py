"""Shared fixtures. Markers: `gpu` = needs an MI355X (run on the GPU box with -m gpu)."""
import ctypes
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def _build_oracle():
    so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    return so


@pytest.fixture(scope="session")
def oracle():
    """The CPU restatement of src/ether_fcs.c (test infrastructure only)."""
    L = ctypes.CDLL(_build_oracle())
    u64, u32, vp, i32 = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int
    L.oracle_ether_fcs.restype = u32
    L.oracle_ether_fcs.argtypes = [vp, ctypes.c_size_t]
    L.oracle_crc32_fast.restype = u32
    L.oracle_crc32_fast.argtypes = [vp, ctypes.c_size_t]
    L.oracle_fcs_batch.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, i32]
    L.oracle_fcs_fixed.argtypes = [vp, ctypes.c_size_t, u32, ctypes.c_size_t, vp, i32, i32]
    L.oracle_time_fixed.restype = ctypes.c_double
    L.oracle_time_fixed.argtypes = [vp, ctypes.c_size_t, u32, ctypes.c_size_t, vp, i32, i32]
    L.oracle_xorshift64_fill.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(u64)]
    L.oracle_splitmix_fill.argtypes = [vp, ctypes.c_size_t, u64, u64]
    L.oracle_splitmix_digest.argtypes = [u64, vp, vp, u64, u32, u64, i32, ctypes.POINTER(u32), ctypes.POINTER(u64)]
    L.oracle_selfcheck.restype = i32
    return L


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(GOLDEN, vec["arena"]), "rb") as f:
        arena = f.read()
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        kat = json.load(f)
    return {"vectors": vec, "arena": arena, "kat": kat}


def splitmix_digest(oracle, seed, n, stride=0, flen=0, off=None, lengths=None, threads=16):
    """(XOR, 64-bit sum) of the CRCs of a whole splitmix batch, computed by the oracle over `threads`
    host threads without materialising the frames (frame i = stream bytes [off_i, +len_i), or
    [i * stride, +flen)). 16 threads: one GPU box's CPU share."""
    x, s = ctypes.c_uint32(0), ctypes.c_uint64(0)
    oracle.oracle_splitmix_digest(seed, None if off is None else off.ctypes.data,
                                  None if lengths is None else lengths.ctypes.data, stride, flen, n, threads,
                                  ctypes.byref(x), ctypes.byref(s))
    return x.value, s.value


@pytest.fixture(params=["quarter", "windowed"])
def var_kernel(request):
    """Run a variable-length test through both var kernels (identical results required):
    quarter = one quarter-wave per frame (small batches), windowed = 64-frame windows."""
    import nstack_amd as na
    old = na.set_var_threshold((1 << 63) if request.param == "quarter" else 0)
    yield request.param
    na.set_var_threshold(old)


@pytest.fixture(scope="session")
def inet_oracle():
    """CPU restatement of ip_checksum / tcp_checksum / udp_checksum (test infrastructure only)."""
    so = os.path.join(ROOT, "oracle", "_build", "liboracle_inet.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    L = ctypes.CDLL(so)
    u16, u32, vp, sz = ctypes.c_uint16, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t
    L.oracle_ip_checksum.restype = u16
    L.oracle_ip_checksum.argtypes = [vp, sz]
    L.oracle_tcp_checksum.restype = u16
    L.oracle_tcp_checksum.argtypes = [u32, u32, vp, sz]
    L.oracle_udp_checksum.restype = u16
    L.oracle_udp_checksum.argtypes = [vp, sz, u32, u32]
    L.oracle_inet_batch.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, sz]
    u64 = ctypes.c_uint64
    L.oracle_inet_splitmix_digest.argtypes = [ctypes.c_int, u64, vp, vp, u64, u32, vp, u64, ctypes.c_int,
                                              ctypes.POINTER(u64), ctypes.POINTER(u64)]
    return L


@pytest.fixture(scope="session")
def inet_golden():
    with open(os.path.join(GOLDEN, "inet_vectors.json")) as f:
        vec = json.load(f)
    with open(os.path.join(GOLDEN, vec["arena"]), "rb") as f:
        vec["arena_bytes"] = f.read()
    return vec
