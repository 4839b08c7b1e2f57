"""Internet-checksum oracle (oracle/inet_oracle.c, a restatement of src/ip.c:39-62,
src/tcp.c:167-213, src/udp.c:136-174) pinned against published known answers and the
independent RFC 1071 witness in tests/golden/make_inet_golden.py. The reference's own functions
could not be built here, so parity with them is pinned only through these."""
import random
import struct

import numpy as np
import pytest

from golden.make_inet_golden import witness


def _one(o, mode, b, src=0, dst=0):
    if mode == "ip":
        return o.oracle_ip_checksum(b, len(b))
    if mode == "tcp":
        return o.oracle_tcp_checksum(src, dst, b, len(b))
    return o.oracle_udp_checksum(b, len(b), src, dst)


def test_known_answers(inet_oracle, inet_golden):
    for k in inet_golden["kat"]:
        b = bytes.fromhex(k["hex"])
        assert struct.pack("<H", _one(inet_oracle, k["mode"], b)).hex() == k["expect_wire"], k


def test_golden_vectors(inet_oracle, inet_golden):
    a = inet_golden["arena_bytes"]
    for r in inet_golden["packets"]:
        b = a[r["off"]:r["off"] + r["len"]]
        assert _one(inet_oracle, r["mode"], b, r["src"], r["dst"]) == r["expect"], r["tag"]


def test_filled_headers_verify_to_zero(inet_oracle, inet_golden):
    a = inet_golden["arena_bytes"]
    filled = [r for r in inet_golden["packets"] if r["tag"] == "ip_hdr_filled"]
    assert filled
    for r in filled:
        assert inet_oracle.oracle_ip_checksum(a[r["off"]:r["off"] + r["len"]], r["len"]) == 0


@pytest.mark.parametrize("mode", ["ip", "tcp", "udp"])
def test_random_against_witness(inet_oracle, mode):
    rng = random.Random(7)
    for _ in range(2000):
        n = rng.randrange(0, 3000)
        b = rng.randbytes(n)
        s, d = rng.getrandbits(32), rng.getrandbits(32)
        assert _one(inet_oracle, mode, b, s, d) == witness(mode, b, s, d)


def test_tcp_segment_with_checksum_in_place_verifies(inet_oracle):
    """tcp_hton (src/tcp.c:298-299) zeroes the field, then stores the checksum; the receive-side
    check (src/tcp.c:510, disabled there) expects 0 over the filled segment."""
    rng = random.Random(3)
    for n in (20, 21, 40, 1480, 1481):
        seg = bytearray(rng.randbytes(n))
        seg[16:18] = b"\0\0"
        s, d = rng.getrandbits(32), rng.getrandbits(32)
        c = inet_oracle.oracle_tcp_checksum(s, d, bytes(seg), n)
        seg[16:18] = struct.pack("<H", c)
        assert inet_oracle.oracle_tcp_checksum(s, d, bytes(seg), n) == 0


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_splitmix_digest_matches_batch(inet_oracle, oracle, mode):
    """The threaded digest (packets regenerated from the splitmix stream) equals the digest of the
    per-packet restatement over the same bytes (fcs_oracle.c's oracle_splitmix_fill)."""
    import ctypes
    rng = np.random.default_rng(mode + 40)
    n = 3001
    ln = rng.choice([0, 1, 20, 64, 576, 1500, 1518, 4000], n).astype(np.uint32)
    off = np.concatenate([[3], 3 + np.cumsum(ln)[:-1]]).astype(np.uint64)
    total = int(off[-1] + ln[-1])
    arena = np.empty(total, dtype=np.uint8)
    oracle.oracle_splitmix_fill(arena.ctypes.data, total, 77, 0)
    addr = rng.integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    out = np.empty(n, dtype=np.uint16)
    inet_oracle.oracle_inet_batch(mode, arena.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                  addr.ctypes.data if mode else None, out.ctypes.data, n)
    s, w = ctypes.c_uint64(), ctypes.c_uint64()
    inet_oracle.oracle_inet_splitmix_digest(mode, 77, off.ctypes.data, ln.ctypes.data, 0, 0,
                                            addr.ctypes.data if mode else None, n, 4, ctypes.byref(s), ctypes.byref(w))
    idx = np.arange(n, dtype=np.uint64) & np.uint64(0xFFFF)
    assert s.value == int(out.astype(np.uint64).sum())
    assert w.value == int((out.astype(np.uint64) * idx).sum())
