"""Frame batches on disk (include/nstack_pcap.h): classic pcap <-> batch layout.

Host-only code, so it runs in the CPU suite. Files are built byte by byte here with struct (the
pcap format as published by libpcap: 24-byte global header, 16-byte record headers), in both
byte orders and both timestamp resolutions, and the library's reader and writer are checked
against them.
"""
import os
import struct

import numpy as np
import pytest

import nstack_amd as na


def build_pcap(records, endian="<", magic=0xA1B2C3D4, linktype=1, snaplen=65535, orig=None):
    out = struct.pack(endian + "IHHiIII", magic, 2, 4, 0, 0, snaplen, linktype)
    for i, r in enumerate(records):
        o = len(r) if orig is None else orig[i]
        out += struct.pack(endian + "IIII", i, 0, len(r), o) + r
    return out


@pytest.fixture
def frames():
    rng = np.random.default_rng(5)
    return [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in [0, 1, 60, 64, 1514, 1518, 9000, 3]]


@pytest.mark.parametrize("endian,magic", [("<", 0xA1B2C3D4), (">", 0xA1B2C3D4), ("<", 0xA1B23C4D), (">", 0xA1B23C4D)])
def test_read_both_byte_orders_and_resolutions(tmp_path, frames, endian, magic):
    p = tmp_path / "x.pcap"
    p.write_bytes(build_pcap(frames, endian, magic, linktype=1))
    assert na.pcap_scan(str(p)) == (len(frames), sum(map(len, frames)), 1, 0)
    arena, off, ln, lt = na.pcap_read(str(p))
    assert lt == 1 and len(off) == len(frames)
    for i, f in enumerate(frames):
        assert ln[i] == len(f) and arena[int(off[i]):int(off[i]) + len(f)].tobytes() == f


def test_write_read_round_trip(tmp_path, frames):
    arena = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    ln = np.array([len(f) for f in frames], dtype=np.uint32)
    off = np.zeros(len(frames), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    p = tmp_path / "rt.pcap"
    na.pcap_write(str(p), arena, off, ln, linktype=1)
    raw = p.read_bytes()
    assert raw[:24] == build_pcap([], "<", 0xA1B2C3D4)[:24]
    a2, o2, l2, lt = na.pcap_read(str(p))
    assert lt == 1 and np.array_equal(l2, ln) and a2.tobytes() == arena.tobytes()


def test_truncated_records_are_counted(tmp_path):
    recs = [b"\x01" * 100, b"\x02" * 64]
    p = tmp_path / "t.pcap"
    p.write_bytes(build_pcap(recs, orig=[1518, 64], snaplen=100))
    assert na.pcap_scan(str(p)) == (2, 164, 1, 1)


def test_errors(tmp_path):
    lib = na.load()
    assert lib.fcs_pcap_scan(os.fsencode(str(tmp_path / "missing.pcap")), None, None, None, None) == -2
    ng = tmp_path / "x.pcapng"
    ng.write_bytes(struct.pack("<III", 0x0A0D0D0A, 28, 0x1A2B3C4D) + b"\0" * 16)
    assert lib.fcs_pcap_scan(os.fsencode(str(ng)), None, None, None, None) == -93   # -EPROTONOSUPPORT
    bad = tmp_path / "bad.pcap"
    bad.write_bytes(b"not a pcap file at all....")
    assert lib.fcs_pcap_scan(os.fsencode(str(bad)), None, None, None, None) == -22
    cut = tmp_path / "cut.pcap"
    cut.write_bytes(build_pcap([b"\x05" * 200])[:-50])
    with pytest.raises(na.FcsError):
        na.pcap_read(str(cut))
    small = np.zeros(10, dtype=np.uint8)
    off = np.zeros(1, dtype=np.uint64)
    ln = np.zeros(1, dtype=np.uint32)
    p = tmp_path / "big.pcap"
    p.write_bytes(build_pcap([b"\x07" * 64]))
    assert lib.fcs_pcap_read(os.fsencode(str(p)), small.ctypes.data, 10, off.ctypes.data, ln.ctypes.data, 1) == -28


def test_edge_files(tmp_path):
    """Empty file, header only, and a record header cut short (the mmap parser's bounds)."""
    lib = na.load()
    e = tmp_path / "empty.pcap"
    e.write_bytes(b"")
    assert lib.fcs_pcap_scan(os.fsencode(str(e)), None, None, None, None) == -22
    h = tmp_path / "hdr.pcap"
    h.write_bytes(build_pcap([]))
    assert na.pcap_scan(str(h)) == (0, 0, 1, 0)
    c = tmp_path / "cuthdr.pcap"
    c.write_bytes(build_pcap([b"\x01" * 30]) + b"\x00" * 10)
    assert lib.fcs_pcap_scan(os.fsencode(str(c)), None, None, None, None) == -22


def test_large_capture_parallel_copy(tmp_path):
    """Over 64 MiB of records the read copies them on several threads, split by bytes: every
    record must land at its packed offset intact (158 MB, lengths 60..1518: two threads)."""
    rng = np.random.default_rng(9)
    n = 200000
    lens = rng.integers(60, 1519, n).astype(np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = rng.integers(0, 256, int(off[-1] + lens[-1]), dtype=np.uint8)
    p = tmp_path / "large.pcap"
    na.pcap_write(str(p), arena, off, lens)
    got, o2, l2, lt = na.pcap_read(str(p))
    assert lt == 1 and np.array_equal(l2, lens) and np.array_equal(o2, off)
    assert np.array_equal(got, arena)
