"""Internet-checksum oracle (oracle/inet_oracle.c, a restatement of src/ip.c:39-62,
src/tcp.c:167-213, src/udp.c:136-174) pinned against published known answers and the
independent RFC 1071 witness in tests/golden/make_inet_golden.py. The reference's own functions
could not be built here, so parity with them is pinned only through these."""
import random
import struct

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
