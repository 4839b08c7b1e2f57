"""The library's own host CRC (fcs_host_crc32, nstack_amd/csrc/fcs_host_crc.cpp): what the host forms
answer a failed GPU step with and what the TX queue computes batches below its GPU minimum with
(nstack_txq.h, fcs_txq_set_host_max). Each of its forms (carry-less folding 128 or 512 bits wide,
slice-by-16 tables) must give the reference's ether_fcs (src/ether_fcs.c:4-19) on the golden vectors
(generated from the compiled reference), the known answers, and every length and alignment around
the folding's 16-, 64- and 256-byte steps, checked against the oracle and zlib. No GPU is involved."""
import ctypes
import os
import random
import subprocess
import sys
import zlib

import pytest

import nstack_amd as na

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _crc(buf: bytes) -> int:
    return na.load().fcs_host_crc32(buf, len(buf))


def test_known_answers(golden):
    assert _crc(b"123456789") == 0xCBF43926
    for k in golden["kat"]["cases"]:
        data = bytes.fromhex(k["hex"]) if k["hex"] is not None else bytes([k["fill"]]) * k["len"]
        assert _crc(data) == k["crc"], k["name"]
        # the residue: a frame followed by its little-endian FCS (src/linux/ether.c:263)
        assert _crc(data + _crc(data).to_bytes(4, "little")) == golden["kat"]["residue"]


def test_golden_vectors(golden):
    arena = golden["arena"]
    for f in golden["vectors"]["frames"]:
        o, n = f["off"], f["len"]
        assert _crc(arena[o:o + n]) == f["crc"], (o, n)


def test_every_length_and_alignment(oracle):
    r = random.Random(7)
    buf = bytes(r.randrange(256) for _ in range(4096 + 64))
    raw = ctypes.create_string_buffer(buf, len(buf))
    L = na.load()
    for n in list(range(0, 600)) + [767, 768, 769, 1023, 1024, 1025, 1279, 1280, 1281, 1514, 1518, 1522, 2047,
                                     2048, 4000]:
        for a in range(16):
            p = ctypes.addressof(raw) + a
            want = oracle.oracle_ether_fcs(p, n)
            assert L.fcs_host_crc32(p, n) == want, (n, a)
            assert want == zlib.crc32(buf[a:a + n])


def test_large_buffers_against_zlib():
    r = random.Random(11)
    for n in (65536, 65537, 1 << 20, (1 << 20) + 13, 9000 * 7 + 5):
        b = r.randbytes(n)
        assert _crc(b) == zlib.crc32(b), n


@pytest.mark.parametrize("form", ["tables", "pclmul"])
def test_narrower_forms_match(form):
    """NSTACK_FCS_HOST_CRC=tables: the slice-by-16 form alone (CPUs without PCLMULQDQ); =pclmul: the
    128-bit folding alone (CPUs without AVX-512 VPCLMULQDQ). The default run above takes the widest
    form the CPU has."""
    code = ("import random, zlib, nstack_amd as na\n"
            "L = na.load(); r = random.Random(3)\n"
            "bad = [n for n in list(range(0, 600)) + [1514, 1518, 9000, 100003]\n"
            "       for b in [r.randbytes(n)] if L.fcs_host_crc32(b, n) != zlib.crc32(b)]\n"
            "print(len(bad))\n")
    env = dict(os.environ, NSTACK_FCS_HOST_CRC=form)
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.strip().splitlines()[-1] == "0"
