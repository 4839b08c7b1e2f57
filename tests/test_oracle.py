"""The oracle is pinned before it is trusted: against the golden fixtures generated from the
reference's own src/ether_fcs.c (tests/golden/make_golden.py), zlib, and SURVEY §8c anchors."""
import ctypes
import os
import random
import struct
import zlib

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kat_bytes(case):
    if case["hex"] is not None:
        return bytes.fromhex(case["hex"])
    return bytes([case["fill"]]) * case["len"]


def test_selfcheck(oracle):
    assert oracle.oracle_selfcheck() == 0


def test_known_answers(oracle, golden):
    for case in golden["kat"]["cases"]:
        b = _kat_bytes(case)
        assert oracle.oracle_ether_fcs(b, len(b)) == case["crc"], case["name"]
        assert oracle.oracle_crc32_fast(b, len(b)) == case["crc"], case["name"]
    assert golden["kat"]["residue"] == 0x2144DF1C


def test_golden_vectors(oracle, golden):
    arena = golden["arena"]
    for fr in golden["vectors"]["frames"]:
        b = arena[fr["off"]:fr["off"] + fr["len"]]
        assert oracle.oracle_ether_fcs(b, len(b)) == fr["crc"]
        assert oracle.oracle_crc32_fast(b, len(b)) == fr["crc"]
        assert zlib.crc32(b) == fr["crc"]


def test_residue_property(oracle):
    rng = random.Random(3)
    for n in list(range(0, 70)) + [1514, 1518, 9000]:
        b = bytes(rng.randrange(256) for _ in range(n))
        c = oracle.oracle_ether_fcs(b, n)
        b2 = b + struct.pack("<I", c)
        assert oracle.oracle_ether_fcs(b2, n + 4) == 0x2144DF1C


def test_random_vs_zlib(oracle):
    rng = random.Random(11)
    for _ in range(2000):
        n = rng.randrange(0, 2000)
        b = os.urandom(n)
        assert oracle.oracle_ether_fcs(b, n) == zlib.crc32(b)
        assert oracle.oracle_crc32_fast(b, n) == zlib.crc32(b)


def test_survey_dataset_digest(oracle, golden):
    """xorshift64 seed 42, 1 M x 1518 B packed -> XOR 0x600A585E."""
    d = golden["vectors"]["xorshift_1m_1518"]
    n, L = d["frames"], d["len"]
    buf = np.empty(n * L, dtype=np.uint8)
    st = ctypes.c_uint64(d["seed"])
    oracle.oracle_xorshift64_fill(buf.ctypes.data, buf.size, ctypes.byref(st))
    assert bytes(buf[:4]).hex() == d["first_bytes"]
    out = np.empty(n, dtype=np.uint32)
    oracle.oracle_fcs_fixed(buf.ctypes.data, L, L, n, out.ctypes.data, 1, 8)
    assert int(np.bitwise_xor.reduce(out)) == d["xor"] == 0x600A585E
    assert int(out.astype(np.uint64).sum()) & (2**64 - 1) == d["sum64"]
    assert int(out[0]) == d["first"] and int(out[-1]) == d["last"]
    # nibble restatement on a slice agrees with the fast form
    ref = np.empty(4096, dtype=np.uint32)
    oracle.oracle_fcs_fixed(buf.ctypes.data, L, L, 4096, ref.ctypes.data, 0, 1)
    assert np.array_equal(ref, out[:4096])


def test_splitmix_generator_matches_python(oracle):
    def splitmix(x):
        x = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return x ^ (x >> 31)
    seed, off, n = 1234, 13, 77
    buf = np.empty(n, dtype=np.uint8)
    oracle.oracle_splitmix_fill(buf.ctypes.data, n, seed, off)
    exp = bytes((splitmix(seed + ((off + i) >> 3)) >> (8 * ((off + i) & 7))) & 0xFF for i in range(n))
    assert bytes(buf) == exp


@pytest.mark.skipif(not os.path.exists("/root/reference/src/ether_fcs.c"),
                    reason="reference sources only exist in the build container")
def test_oracle_matches_compiled_reference(oracle):
    """oracle/_ref/libref_fcs.so is /root/reference/src/ether_fcs.c built by oracle/Makefile."""
    import subprocess
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_fcs.so"))
    ref.ether_fcs.restype = ctypes.c_uint32
    ref.ether_fcs.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    rng = random.Random(7)
    for _ in range(3000):
        n = rng.randrange(0, 9100)
        b = os.urandom(n)
        assert ref.ether_fcs(b, n) == oracle.oracle_ether_fcs(b, n)


def test_bench_host_generator_matches_device_generator_restatement(oracle):
    """bench.py re-creates sampled frames with a numpy splitmix64 (no oracle in its timed leg);
    it must equal the oracle's restatement of the device generator at any offset."""
    import numpy as np
    import bench
    for seed, off, n in ((0x4E535441434B, 0, 1518), (0x4E535441434B, 1518 * 12345 + 3, 1518), (7, 5, 1), (1, 8, 64)):
        buf = np.empty(n, dtype=np.uint8)
        oracle.oracle_splitmix_fill(buf.ctypes.data, n, seed, off)
        assert np.array_equal(bench.splitmix_bytes(seed, off, n), buf)


@pytest.mark.parametrize("fixed", [(1518, 1518, 3000), (9000, 9001, 200), (70000, 70000, 5), (64, 100, 4000)])
def test_splitmix_digest_fixed_matches_zlib(oracle, fixed):
    """The whole-batch digest the BASELINE-size GPU tests compare against (XOR and 64-bit sum of every
    frame's CRC, frames regenerated from the splitmix stream on the fly) equals zlib's over the same
    bytes; frames over 64 KiB take the piecewise path."""
    from conftest import splitmix_digest
    L, stride, n = fixed
    buf = np.empty(L, dtype=np.uint8)
    x, s = 0, 0
    for i in range(n):
        oracle.oracle_splitmix_fill(buf.ctypes.data, L, 31, i * stride)
        c = zlib.crc32(buf.tobytes())
        x ^= c
        s += c
    assert splitmix_digest(oracle, 31, n, stride=stride, flen=L, threads=3) == (x, s & ((1 << 64) - 1))


def test_splitmix_digest_var_matches_zlib(oracle):
    from conftest import splitmix_digest
    rng = np.random.default_rng(12)
    ln = rng.choice(np.array([0, 1, 64, 576, 1518, 9000], dtype=np.uint32), 3000)
    off = np.zeros(len(ln), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + 5)
    x, s = 0, 0
    for o, L in zip(off, ln):
        buf = np.empty(int(L), dtype=np.uint8)
        oracle.oracle_splitmix_fill(buf.ctypes.data, int(L), 8, int(o))
        c = zlib.crc32(buf.tobytes())
        x ^= c
        s += c
    assert splitmix_digest(oracle, 8, len(ln), off=off, lengths=ln, threads=5) == (x, s & ((1 << 64) - 1))
