"""pcap-driven batches on the GPU: fixtures and captures through the engine.

The golden vectors (generated from the compiled reference src/ether_fcs.c, tests/golden/) are
written as a pcap, read back into the batch layout and checksummed on the GPU; frames built in
ether_send's TX layout (src/linux/ether.c:222-263) are written as a capture with FCS trailers and
verified by the RX residue check.
"""
import struct

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    na.load()
    return torch.device("cuda:0")


def test_golden_vectors_through_pcap(dev, var_kernel, golden, tmp_path):
    fr = golden["vectors"]["frames"]
    arena = np.frombuffer(golden["arena"], dtype=np.uint8)
    off = np.array([f["off"] for f in fr], dtype=np.uint64)
    ln = np.array([f["len"] for f in fr], dtype=np.uint32)
    p = tmp_path / "golden.pcap"
    na.pcap_write(str(p), arena, off, ln)
    a2, o2, l2, lt = na.pcap_read(str(p))
    out = np.zeros(len(l2), dtype=np.uint32)
    na.batch_host(a2, a2.nbytes, o2, l2, out, len(l2))
    assert np.array_equal(out, np.array([f["crc"] for f in fr], dtype=np.uint32))


def test_capture_with_fcs_verifies(dev, oracle, tmp_path):
    rng = np.random.default_rng(17)
    frames = []
    for _ in range(3000):
        bsize = int(rng.integers(0, 1501))
        size = 14 + max(bsize, 56) + 4
        body = rng.integers(0, 256, size - 4, dtype=np.uint8)
        body[14 + bsize:] = 0
        fcs = oracle.oracle_ether_fcs(body.ctypes.data, size - 4)
        frames.append(body.tobytes() + struct.pack("<I", fcs))
    bad = set(int(x) for x in rng.choice(len(frames), 40, replace=False))
    for i in bad:
        b = bytearray(frames[i])
        b[int(rng.integers(0, len(b)))] ^= 0x80
        frames[i] = bytes(b)
    arena = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    ln = np.array([len(f) for f in frames], dtype=np.uint32)
    off = np.zeros(len(frames), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    p = tmp_path / "rx.pcap"
    na.pcap_write(str(p), arena, off, ln)
    a2, o2, l2, _ = na.pcap_read(str(p))
    ok = np.zeros(len(l2), dtype=np.uint8)
    assert na.verify_host(a2, a2.nbytes, o2, l2, ok, len(l2)) == len(bad)
    assert set(np.nonzero(ok == 0)[0].tolist()) == bad


def test_add_fcs_to_a_capture(dev, oracle, tmp_path):
    """tools/pcap_fcs.py --add-fcs: a capture without trailers (as veth delivers it) becomes the
    capture the wire would carry: every frame followed by ether_send's FCS (GPU TX mode), which
    the residue check then accepts and which matches the oracle byte for byte."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "pcap_fcs", os.path.join(os.path.dirname(__file__), "..", "tools", "pcap_fcs.py"))
    tool = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tool)
    rng = np.random.default_rng(21)
    ln = rng.integers(60, 1515, 500).astype(np.uint32)
    off = np.zeros(len(ln), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    arena = rng.integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    src, dst = tmp_path / "plain.pcap", tmp_path / "fcs.pcap"
    na.pcap_write(str(src), arena, off, ln)
    a1, o1, l1, lt = na.pcap_read(str(src))
    tool.add_fcs(a1, o1, l1, str(dst), lt)
    a2, o2, l2, _ = na.pcap_read(str(dst))
    assert np.array_equal(l2, ln + 4)
    ok = np.zeros(len(l2), dtype=np.uint8)
    assert na.verify_host(a2, a2.nbytes, o2, l2, ok, len(l2)) == 0 and ok.all()
    for i in rng.integers(0, len(ln), 40):
        o, L = int(o2[i]), int(ln[i])
        assert a2[o:o + L].tobytes() == arena[int(off[i]):int(off[i]) + L].tobytes()
        c = oracle.oracle_ether_fcs(arena[int(off[i]):].ctypes.data, L)
        assert a2[o + L:o + L + 4].tobytes() == struct.pack("<I", c)
