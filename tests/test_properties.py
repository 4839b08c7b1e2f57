"""Property-based checks (hypothesis) of the host-side pieces that need no GPU: the oracles against
independent witnesses, the pcap reader/writer round trip, and the TX queue's ether_send size rule.
Example counts are kept small so the CPU suite stays fast; the seeds are derandomized so a failure
reproduces."""
import struct
import zlib

import numpy as np
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

import nstack_amd as na  # noqa: E402
from golden.make_inet_golden import witness  # noqa: E402

FAST = settings(max_examples=150, deadline=None, derandomize=True)


@FAST
@given(st.binary(min_size=0, max_size=4096))
def test_fcs_oracle_is_crc32(oracle, data):
    """src/ether_fcs.c:4-19 restated == CRC-32/ISO-HDLC (zlib), both oracle variants."""
    assert oracle.oracle_ether_fcs(data, len(data)) == zlib.crc32(data)
    assert oracle.oracle_crc32_fast(data, len(data)) == zlib.crc32(data)


@FAST
@given(st.binary(min_size=0, max_size=2048))
def test_fcs_residue(oracle, data):
    """ether_send stores the FCS little-endian after the covered bytes (src/linux/ether.c:263);
    the whole frame then always leaves the CRC-32 residue 0x2144DF1C."""
    frame = data + struct.pack("<I", oracle.oracle_ether_fcs(data, len(data)))
    assert oracle.oracle_ether_fcs(frame, len(frame)) == 0x2144DF1C


@FAST
@given(st.sampled_from(["ip", "tcp", "udp"]), st.binary(min_size=0, max_size=3000),
       st.integers(0, 2**32 - 1), st.integers(0, 2**32 - 1))
def test_inet_oracle_matches_witness(inet_oracle, mode, data, src, dst):
    n = len(data)
    if mode == "ip":
        got = inet_oracle.oracle_ip_checksum(data, n)
    elif mode == "tcp":
        got = inet_oracle.oracle_tcp_checksum(src, dst, data, n)
    else:
        got = inet_oracle.oracle_udp_checksum(data, n, src, dst)
    assert got == witness(mode, data, src, dst)


@FAST
@given(st.binary(min_size=20, max_size=60).map(bytearray))
def test_ip_header_with_its_checksum_verifies(inet_oracle, hdr):
    """ip_hton zeroes ip_csum and stores ip_checksum there (src/ip.c:79-80); the receive-side
    check (src/ip.c:151) then sees 0."""
    hdr[10:12] = b"\0\0"
    c = inet_oracle.oracle_ip_checksum(bytes(hdr), len(hdr))
    hdr[10:12] = struct.pack("<H", c)
    assert inet_oracle.oracle_ip_checksum(bytes(hdr), len(hdr)) == 0


@settings(max_examples=40, deadline=None, derandomize=True)
@given(st.lists(st.binary(min_size=0, max_size=2000), min_size=0, max_size=20), st.sampled_from([1, 101, 105]))
def test_pcap_round_trip(tmp_path_factory, frames, linktype):
    """fcs_pcap_write then fcs_pcap_read reproduce every frame byte for byte, in order."""
    p = tmp_path_factory.mktemp("pc") / "rt.pcap"
    arena = np.frombuffer(b"".join(frames) or b"\0", dtype=np.uint8).copy()
    off = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64) if frames else np.zeros(0, np.uint64)
    ln = np.array([len(f) for f in frames], dtype=np.uint32)
    na.pcap_write(str(p), arena, off, ln, linktype)
    n, b, lt, trunc = na.pcap_scan(str(p))
    assert (n, b, lt, trunc) == (len(frames), sum(map(len, frames)), linktype, 0)
    if frames:
        a2, o2, l2, _ = na.pcap_read(str(p))
        for i, f in enumerate(frames):
            assert l2[i] == len(f) and a2[int(o2[i]):int(o2[i]) + len(f)].tobytes() == f


@settings(max_examples=60, deadline=None, derandomize=True)
@given(st.integers(0, 3000))
def test_txq_size_rule(bsize):
    """ether_send: frame_size = 14 + max(bsize, 56) + 4 (src/linux/ether.c:222-224); more than
    1518 is -EMSGSIZE before anything is queued (:234-237)."""
    import socket
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    try:
        with na.TxQueue(bytes([2, 0, 0, 0, 0, 1]), a.fileno(), max_batch=4) as q:
            fs = 14 + max(bsize, 56) + 4
            if fs > 1518:
                assert q.send_async(bytes(6), 0x0800, bytes(bsize)) == -90
                assert q.stats() == (0, 0, 0)
            else:
                assert q.send_async(bytes(6), 0x0800, bytes(bsize)) == fs
    finally:
        a.close(), b.close()
