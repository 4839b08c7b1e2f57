"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bit-exact is the only bar (integer CRC). Sizes here finish in seconds on the oracle; the
BASELINE-size run (64 M x 1518 B) is checked through size-independent properties: sampled frames
against the oracle, shard consistency (two half launches == one launch), determinism, and the
CRC residue of every frame written in TX mode.
"""
import ctypes
import os
import random
import struct
import threading
import zlib

import numpy as np
import pytest

import nstack_amd as na
from conftest import splitmix_digest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    na.load()
    return torch.device("cuda:0")


def to_dev(arr: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(arr)).to(dev)


def oracle_fixed(oracle, host: np.ndarray, stride, L, n, fast=1):
    out = np.empty(n, dtype=np.uint32)
    oracle.oracle_fcs_fixed(host.ctypes.data, stride, L, n, out.ctypes.data, fast, 16)
    return out


def oracle_var(oracle, arena: np.ndarray, off, ln, fast=1):
    out = np.empty(len(off), dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    oracle.oracle_fcs_batch(arena.ctypes.data, off.ctypes.data, ln.ctypes.data, out.ctypes.data, len(off), fast)
    return out


def run_var(dev, arena_np: np.ndarray, off, ln):
    arena = to_dev(arena_np, dev)
    o = to_dev(np.asarray(off, dtype=np.uint64).view(np.int64), dev)
    l_ = to_dev(np.asarray(ln, dtype=np.uint32).view(np.int32), dev)
    out = torch.empty(len(off), dtype=torch.int32, device=dev)
    na.batch_dev(arena, arena_np.nbytes, o, l_, out, len(off))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def run_fixed(dev, base_t, stride, L, n):
    out = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(base_t, stride, L, n, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


# ---------------------------------------------------------------- fixtures (golden, KAT)
def test_golden_vectors_var(dev, var_kernel, golden):
    arena = np.frombuffer(golden["arena"], dtype=np.uint8).copy()
    fr = golden["vectors"]["frames"]
    got = run_var(dev, arena, [f["off"] for f in fr], [f["len"] for f in fr])
    exp = np.array([f["crc"] for f in fr], dtype=np.uint32)
    assert np.array_equal(got, exp)


def test_golden_vectors_fixed_one_by_one(dev, golden):
    arena = np.frombuffer(golden["arena"], dtype=np.uint8).copy()
    a = to_dev(arena, dev)
    for f in golden["vectors"]["frames"][::7]:
        got = run_fixed(dev, a.data_ptr() + f["off"], max(f["len"], 1), f["len"], 1)
        assert int(got[0]) == f["crc"], f


def test_known_answers(dev, var_kernel, golden):
    for case in golden["kat"]["cases"]:
        b = bytes.fromhex(case["hex"]) if case["hex"] is not None else bytes([case["fill"]]) * case["len"]
        arr = np.frombuffer(b + b"\0" * 8, dtype=np.uint8).copy()
        got = run_var(dev, arr, [0], [len(b)])
        assert int(got[0]) == case["crc"], case["name"]


def test_dropin_ether_fcs(dev, golden):
    assert na.ether_fcs(b"123456789") == 0xCBF43926
    assert na.ether_fcs(b"") == 0
    arena = golden["arena"]
    for f in golden["vectors"]["frames"][::11]:
        assert na.ether_fcs(arena[f["off"]:f["off"] + f["len"]]) == f["crc"]


def test_dropin_every_length(dev, golden):
    """The drop-in takes frames of up to 1536 B through the single-frame kernel (the frame rides in
    the kernel arguments) and longer ones through the staged path: every length 0..1600 from
    several source alignments, the golden known answers, and the residue of a frame with its
    own FCS appended, all against zlib (= the reference ether_fcs)."""
    rng = np.random.default_rng(77)
    buf = rng.integers(0, 256, 1700, dtype=np.uint8).tobytes()
    for L in range(0, 1601):
        a = (L * 7) % 13
        b = buf[a:a + L]
        assert na.ether_fcs(b) == zlib.crc32(b), L
    for case in golden["kat"]["cases"]:
        b = bytes.fromhex(case["hex"]) if case["hex"] is not None else bytes([case["fill"]]) * case["len"]
        assert na.ether_fcs(b) == case["crc"], case["name"]
    for L in (60, 1514, 1532):
        f = buf[:L]
        assert na.ether_fcs(f + struct.pack("<I", zlib.crc32(f))) == 0x2144DF1C
    # longer buffers: both sides of the interleaved segment kernel's bound, jumbo, 64 KiB, odd sizes
    big = rng.integers(0, 256, 100020, dtype=np.uint8).tobytes()
    for L in (2285, 2286, 3000, 3049, 9000, 9001, 65536, 100003):
        a = L % 7
        assert na.ether_fcs(big[a:a + L]) == zlib.crc32(big[a:a + L]), L


# ---------------------------------------------------------------- edge lengths / alignment
EDGE = [0, 1, 3, 4, 59, 60, 61, 63, 64, 65, 69, 70, 71, 575, 576, 577, 1487, 1488, 1489,
        1513, 1514, 1515, 1516, 1517, 1518, 1535, 1536, 1537, 3071, 3072, 3073, 8999, 9000]


@pytest.mark.parametrize("L", EDGE)
def test_fixed_edge_lengths_all_alignments(dev, oracle, L):
    n = 4099
    for stride in sorted({max(L, 1), L + 1, L + 2, L + 3, ((L + 63) // 64) * 64 or 64}):
        host = np.random.default_rng(L * 7 + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
        d = to_dev(host, dev)
        for lead in (0, 1, 2, 3):
            nn = n - 1
            got = run_fixed(dev, d.data_ptr() + lead, stride, L, nn)
            exp = oracle_fixed(oracle, host[lead:], stride, L, nn)
            assert np.array_equal(got, exp), (L, stride, lead, int(np.argmax(got != exp)))


def test_frames_touching_allocation_edges(dev, var_kernel, oracle):
    """Frame 0 at the very start and the last frame ending at the very end of the buffer."""
    for L in (1, 5, 70, 1517, 1518, 9000):
        n = 33
        host = np.random.default_rng(L).integers(0, 256, n * L, dtype=np.uint8)
        d = to_dev(host, dev)
        got = run_fixed(dev, d, L, L, n)
        assert np.array_equal(got, oracle_fixed(oracle, host, L, L, n))
        got = run_var(dev, host, [i * L for i in range(n)], [L] * n)
        assert np.array_equal(got, oracle_fixed(oracle, host, L, L, n))


# ---------------------------------------------------------------- variable length
def test_random_lengths_random_offsets(dev, var_kernel, oracle):
    rng = np.random.default_rng(5)
    n = 20000
    ln = rng.integers(0, 9019, n).astype(np.uint32)
    ln[rng.random(n) < 0.05] = 0
    size = int(ln.sum()) + 4 * n + 64
    arena = rng.integers(0, 256, size, dtype=np.uint8)
    off = rng.integers(0, size - 9019, n).astype(np.uint64)  # overlapping, unordered
    got = run_var(dev, arena, off, ln)
    assert np.array_equal(got, oracle_var(oracle, arena, off, ln))


def imix(n, seed):
    counts = [n * 7 // 12, n * 4 // 12]
    counts.append(n - sum(counts))
    ln = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), counts)
    np.random.default_rng(seed).shuffle(ln)
    return ln


def test_imix_packed(dev, var_kernel, oracle):
    ln = imix(120000, 3)
    off = np.zeros(len(ln), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    size = int(off[-1] + ln[-1])
    arena = np.random.default_rng(4).integers(0, 256, size, dtype=np.uint8)
    got = run_var(dev, arena, off, ln)
    assert np.array_equal(got, oracle_var(oracle, arena, off, ln))


def test_jumbo(dev, oracle):
    n, L = 4096, 9000
    host = np.random.default_rng(6).integers(0, 256, n * L, dtype=np.uint8)
    d = to_dev(host, dev)
    assert np.array_equal(run_fixed(dev, d, L, L, n), oracle_fixed(oracle, host, L, L, n))


def test_long_frames(dev, oracle):
    for L in (65536, 100003, 1 << 20):
        n = 7
        host = np.random.default_rng(L).integers(0, 256, n * L + 3, dtype=np.uint8)
        d = to_dev(host, dev)
        got = run_fixed(dev, d.data_ptr() + 3, L, L, n)
        assert np.array_equal(got, oracle_fixed(oracle, host[3:], L, L, n))


# ---------------------------------------------------------------- SURVEY §8c dataset
def test_survey_xorshift_digest(dev, oracle, golden):
    dg = golden["vectors"]["xorshift_1m_1518"]
    n, L = dg["frames"], dg["len"]
    host = np.empty(n * L, dtype=np.uint8)
    st = ctypes.c_uint64(dg["seed"])
    oracle.oracle_xorshift64_fill(host.ctypes.data, host.size, ctypes.byref(st))
    got = run_fixed(dev, to_dev(host, dev), L, L, n)
    assert int(np.bitwise_xor.reduce(got)) == dg["xor"] == 0x600A585E
    assert int(got.astype(np.uint64).sum()) == dg["sum64"]
    assert int(got[0]) == dg["first"] and int(got[-1]) == dg["last"]


# ---------------------------------------------------------------- device generator
def test_device_generator_matches_oracle(dev, oracle):
    for off, nb in ((0, 4096), (5, 1000), (13, 77), (1 << 33, 513)):
        t = torch.zeros(nb + 16, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(t.data_ptr() + 3, nb, 99, off)
        torch.cuda.synchronize()
        h = np.empty(nb, dtype=np.uint8)
        oracle.oracle_splitmix_fill(h.ctypes.data, nb, 99, off)
        got = t.cpu().numpy()
        assert np.array_equal(got[3:3 + nb], h)
        assert not got[:3].any() and not got[3 + nb:].any()


# ---------------------------------------------------------------- BASELINE size (properties)
def _digest(a):
    return int(np.bitwise_xor.reduce(a)), int(a.astype(np.uint64).sum()) & ((1 << 64) - 1)


def test_baseline_size_properties(dev, oracle):
    """64 M x 1518 B (94.9 GiB) in one launch: every frame covered by the XOR and the 64-bit sum of
    all CRCs against the oracle's digest of the same splitmix stream, sampled frames == oracle, two
    half launches == one launch (shard consistency), and a second launch is bit-identical
    (determinism)."""
    free, _ = torch.cuda.mem_get_info()
    n, L = 64 << 20, 1518
    if free < n * L + (4 << 30):
        pytest.skip("not enough HBM")
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, 2026, 0)
    a = run_fixed(dev, arena, L, L, n)
    assert _digest(a) == splitmix_digest(oracle, 2026, n, stride=L, flen=L)
    h = n // 2
    b0 = run_fixed(dev, arena, L, L, h)
    b1 = run_fixed(dev, arena.data_ptr() + h * L, L, L, n - h)
    assert np.array_equal(a, np.concatenate([b0, b1]))
    assert np.array_equal(a, run_fixed(dev, arena, L, L, n))
    rng = np.random.default_rng(1)
    idx = np.unique(np.concatenate([rng.integers(0, n, 3000), [0, 1, n - 2, n - 1]]))
    buf = np.empty(L, dtype=np.uint8)
    for i in idx:
        oracle.oracle_splitmix_fill(buf.ctypes.data, L, 2026, int(i) * L)
        assert int(a[i]) == oracle.oracle_crc32_fast(buf.ctypes.data, L), int(i)
    del arena
    torch.cuda.empty_cache()


def test_baseline_imix_size_properties(dev, oracle):
    """BASELINE configs[2]: 128 M IMIX frames (7:4:1 of 64/576/1518, shuffled, packed; 47.8 GB) in
    one launch of the windowed kernel: every frame covered by the XOR / sum64 digest of all CRCs
    against the oracle's, sampled frames == oracle, the two halves of the frame list launched
    separately == one launch, and a second launch is bit-identical."""
    n = 128 << 20
    rng = np.random.default_rng(2027)
    ln = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), [n * 7 // 12, n * 4 // 12, n - n * 7 // 12 - n * 4 // 12])
    rng.shuffle(ln)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1], dtype=np.uint64, out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    free, _ = torch.cuda.mem_get_info()
    if free < total + 12 * n + (4 << 30):
        pytest.skip("not enough HBM")
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, total, 2027, 0)
    o = to_dev(off.view(np.int64), dev)
    l_ = to_dev(ln.view(np.int32), dev)

    def launch(lo, hi):
        out = torch.empty(hi - lo, dtype=torch.int32, device=dev)
        na.batch_dev(arena, total, o[lo:], l_[lo:], out, hi - lo)
        torch.cuda.synchronize()
        return out.cpu().numpy().view(np.uint32)

    a = launch(0, n)
    assert _digest(a) == splitmix_digest(oracle, 2027, n, off=off, lengths=ln)
    h = n // 2
    assert np.array_equal(a, np.concatenate([launch(0, h), launch(h, n)]))
    assert np.array_equal(a, launch(0, n))
    idx = np.unique(np.concatenate([rng.integers(0, n, 3000), [0, 1, n - 2, n - 1]]))
    buf = np.empty(1518, dtype=np.uint8)
    for i in idx:
        L = int(ln[i])
        oracle.oracle_splitmix_fill(buf.ctypes.data, L, 2027, int(off[i]))
        assert int(a[i]) == oracle.oracle_crc32_fast(buf.ctypes.data, L), int(i)
    del arena, o, l_
    torch.cuda.empty_cache()


def test_more_than_2_32_frames(dev, oracle):
    """2^32 + 1001 one-byte frames in one launch (the flat route without a length array): frame
    indices, window numbers and output offsets past 32 bits. Sampled frames, the frames on both
    sides of index 2^32 and the last frames are checked against the oracle."""
    n = (1 << 32) + 1001
    free, _ = torch.cuda.mem_get_info()
    if free < 5 * n + (4 << 30):
        pytest.skip("not enough HBM")
    arena = torch.empty(n, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n, 2029, 0)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(arena, 1, 1, n, out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(4)
    idx = np.unique(np.concatenate([rng.integers(0, n, 2000), np.arange((1 << 32) - 70, (1 << 32) + 70),
                                    np.arange(n - 70, n), [0, 1]]))
    it = torch.from_numpy(idx.astype(np.int64)).to(dev)
    data = arena[it].cpu().numpy()
    exp = np.array([oracle.oracle_crc32_fast(np.array([b], dtype=np.uint8).ctypes.data, 1) for b in data],
                   dtype=np.uint32)
    assert np.array_equal(out[it].cpu().numpy().view(np.uint32), exp)
    # the same frames as a variable-length batch (offsets and lengths built on the device: 51 GB).
    # torch.arange over more than 2^32 elements returns zeros past index 1023 on this ROCm build of
    # PyTorch, so the offsets are written in pieces of 2^30 and spot-checked before use.
    if free >= 17 * n + (4 << 30):
        off = torch.empty(n, dtype=torch.int64, device=dev)
        for s0 in range(0, n, 1 << 30):
            s1 = min(n, s0 + (1 << 30))
            off[s0:s1] = torch.arange(s0, s1, dtype=torch.int64, device=dev)
        assert np.array_equal(off[it].cpu().numpy(), idx.astype(np.int64))
        ln = torch.ones(n, dtype=torch.int32, device=dev)
        out.zero_()
        na.batch_dev(arena, n, off, ln, out, n)
        torch.cuda.synchronize()
        assert np.array_equal(out[it].cpu().numpy().view(np.uint32), exp)
        del off, ln
    del arena, out
    torch.cuda.empty_cache()


def test_baseline_jumbo_size_properties(dev, oracle):
    """BASELINE configs[3]: 16 M x 9000-B frames (151 GB) in one launch of the interleaved segment
    kernel: every frame covered by the XOR / sum64 digest against the oracle's, sampled frames ==
    oracle, two half launches == one launch, determinism."""
    n, L = 16 << 20, 9000
    free, _ = torch.cuda.mem_get_info()
    if free < n * L + (4 << 30):
        pytest.skip("not enough HBM")
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, 2028, 0)
    a = run_fixed(dev, arena, L, L, n)
    assert _digest(a) == splitmix_digest(oracle, 2028, n, stride=L, flen=L)
    h = n // 2 + 1   # an odd split: the second half starts inside a 4-frame unit of the first launch
    b0 = run_fixed(dev, arena, L, L, h)
    b1 = run_fixed(dev, arena.data_ptr() + h * L, L, L, n - h)
    assert np.array_equal(a, np.concatenate([b0, b1]))
    assert np.array_equal(a, run_fixed(dev, arena, L, L, n))
    rng = np.random.default_rng(3)
    idx = np.unique(np.concatenate([rng.integers(0, n, 2000), [0, 1, n - 2, n - 1]]))
    buf = np.empty(L, dtype=np.uint8)
    for i in idx:
        oracle.oracle_splitmix_fill(buf.ctypes.data, L, 2028, int(i) * L)
        assert int(a[i]) == oracle.oracle_crc32_fast(buf.ctypes.data, L), int(i)
    del arena
    torch.cuda.empty_cache()


# ---------------------------------------------------------------- host-side entry points
def test_fixed_host_and_batch_host(dev, var_kernel, oracle):
    n, L = 300000, 1518
    host = np.random.default_rng(8).integers(0, 256, n * L, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint32)
    na.fixed_host(host, L, L, n, out)
    assert np.array_equal(out, oracle_fixed(oracle, host, L, L, n))
    ln = imix(200000, 9)
    off = np.zeros(len(ln), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    arena = np.random.default_rng(10).integers(0, 256, int(off[-1] + ln[-1]), dtype=np.uint8)
    out2 = np.zeros(len(ln), dtype=np.uint32)
    na.batch_host(arena, arena.nbytes, off, ln, out2, len(ln))
    assert np.array_equal(out2, oracle_var(oracle, arena, off, ln))


@pytest.mark.parametrize("layout", ["packed", "gapped", "shuffled", "jumbo_mix"])
def test_batch_host_many_chunks(dev, oracle, layout):
    """ether_fcs_batch_host over ~450 MB of frames: several 128-MiB pipeline chunks on two streams,
    chunk sizes found by the shrinking min/max/sum pass; shuffled offsets take the gather path
    (span far larger than the bytes), gapped ones are limited by their span."""
    rng = np.random.default_rng(["packed", "gapped", "shuffled", "jumbo_mix"].index(layout) + 40)
    n = 1_200_000
    ln = imix(n, 17).astype(np.uint64)
    if layout == "jumbo_mix":
        ln[rng.integers(0, n, 3000)] = 9000
        ln[rng.integers(0, n, 3000)] = 0
    gap = rng.integers(0, 600, n).astype(np.uint64) if layout == "gapped" else np.zeros(n, dtype=np.uint64)
    start = np.zeros(n, dtype=np.uint64)
    start[1:] = np.cumsum(ln[:-1] + gap[:-1], dtype=np.uint64)
    off = start.copy()
    if layout == "shuffled":
        perm = rng.permutation(n)
        off = start[perm]
        ln = ln[perm]
    total = int((off + ln).max()) + 16
    arena = rng.integers(0, 256, total, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint32)
    na.batch_host(arena, arena.nbytes, off, ln.astype(np.uint32), out, n)
    exp = oracle_var(oracle, arena, off, ln.astype(np.uint32))
    bad = np.nonzero(out != exp)[0]
    assert bad.size == 0, f"{bad.size} frames differ, first {int(bad[0])}"


def test_tx_mode_matches_ether_send_layout(dev, var_kernel, oracle):
    """ether_send (src/linux/ether.c:222-263): frame = hdr + payload + zero pad, FCS over
    frame_size-4 bytes stored little-endian at the end. Batched TX must produce byte-identical
    frames; every frame then satisfies the CRC residue 0x2144DF1C."""
    rng = random.Random(12)
    stride = 1518
    payloads = [rng.randrange(0, 1501) for _ in range(5000)]
    frames = np.zeros((len(payloads), stride), dtype=np.uint8)
    covered = np.zeros(len(payloads), dtype=np.uint32)
    expected = []
    for i, bsize in enumerate(payloads):
        frame_size = 14 + max(bsize, 60 - 4) + 4          # :222-224
        hdr = bytes(rng.randrange(256) for _ in range(12)) + struct.pack(">H", 0x0800)
        body = bytes(rng.randrange(256) for _ in range(bsize))
        f = hdr + body + b"\0" * (frame_size - 14 - bsize)  # :261 zero pad before the FCS
        c = zlib.crc32(f[:frame_size - 4])
        assert c == oracle.oracle_ether_fcs(f, frame_size - 4)
        expected.append(f[:frame_size - 4] + struct.pack("<I", c))  # :262-263
        frames[i, :frame_size - 4] = np.frombuffer(f[:frame_size - 4], dtype=np.uint8)
        covered[i] = frame_size - 4
    na.tx_host(frames, stride, covered, len(payloads))
    for i in range(len(payloads)):
        fs = int(covered[i]) + 4
        assert frames[i, :fs].tobytes() == expected[i]
        assert oracle.oracle_ether_fcs(frames[i].ctypes.data, fs) == 0x2144DF1C


@pytest.mark.parametrize("where,count,maxlen", [("pageable", 3000, 1514), ("pinned", 3000, 1514),
                                               ("pageable", 12000, 1514), ("pinned", 1, 1514), ("pageable", 1, 1536),
                                               ("pinned", 17, 1536), ("pinned", 64, 1536),
                                               ("pinned", 64, 2000), ("pinned", 65, 1536)])
def test_tx_batch_host_offsets(dev, oracle, where, count, maxlen):
    """ether_fcs_tx_batch_host: ether_send's FCS placement (src/linux/ether.c:262-263) over the
    packed-arena layout: frames at arbitrary offsets with gaps, the first at the
    arena's first byte, the FCS written at off + len, nothing else touched. "pinned" runs the
    in-place paths of fcs_host_alloc memory: up to 64 frames of up to 1536 B in the small-batch
    kernel (frame list in its arguments), more frames or longer ones through the mapped-memory
    batch kernel; pageable memory takes the staged pipeline."""
    rng = np.random.default_rng(40 + count + maxlen)
    ln = rng.integers(0, maxlen + 1, count).astype(np.uint32)
    ln[:min(count, 3)] = [maxlen, 0, 1][:min(count, 3)]
    gap = rng.integers(4, 40, count).astype(np.uint64)       # room for the FCS plus slack
    off = np.zeros(count, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gap[:-1])
    nbytes = int(off[-1] + ln[-1] + gap[-1])
    data = rng.integers(0, 256, nbytes, dtype=np.uint8)
    arena = na.host_buffer(nbytes) if where == "pinned" else np.empty(nbytes, dtype=np.uint8)
    try:
        arena[:] = data
        na.tx_batch_host(arena, nbytes, off, ln, count)
        want = data.copy()
        for i in range(count):
            o, L = int(off[i]), int(ln[i])
            c = oracle.oracle_ether_fcs(data[o:o + L].ctypes.data, L) if L else 0
            want[o + L:o + L + 4] = np.frombuffer(struct.pack("<I", c), dtype=np.uint8)
        bad = np.flatnonzero(arena != want)
        assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"
    finally:
        if where == "pinned":
            na.host_free(arena)


def test_tx_in_place_buffers_grow(dev):
    """The in-place TX path keeps mapped length/offset/result arrays sized to the largest batch
    so far; batches that outgrow them (4097 and 9000 frames after 100) must reallocate cleanly,
    with offsets and with a stride, and the next batch must still run."""
    for n in (100, 4097, 9000, 9000, 20):
        a = na.host_buffer(n * 1536)
        try:
            data = np.random.default_rng(n).integers(0, 256, n * 1536, dtype=np.uint8)
            a[:] = data
            ln = np.full(n, 1514, dtype=np.uint32)
            na.tx_batch_host(a, n * 1536, np.arange(n, dtype=np.uint64) * 1536, ln, n)
            for i in (0, n // 2, n - 1):
                f = data[i * 1536:i * 1536 + 1514].tobytes()
                assert a[i * 1536 + 1514:i * 1536 + 1518].tobytes() == struct.pack("<I", zlib.crc32(f)), (n, i)
            a[:] = data
            na.tx_host(a, 1536, ln, n)
            assert a[(n - 1) * 1536 + 1514:(n - 1) * 1536 + 1518].tobytes() == \
                struct.pack("<I", zlib.crc32(data[(n - 1) * 1536:(n - 1) * 1536 + 1514].tobytes()))
        finally:
            na.host_free(a)


def test_tx_batch_host_rejects_fcs_past_arena(dev):
    """The FCS of the last frame must fit inside arena_bytes (-EINVAL, nothing written)."""
    arena = np.zeros(100, dtype=np.uint8)
    with pytest.raises(na.FcsError):
        na.tx_batch_host(arena, 100, np.array([40], dtype=np.uint64), np.array([57], dtype=np.uint32), 1)
    assert not arena.any()


def test_concurrent_callers(dev, oracle):
    """ether_fcs is called from 3-4 threads in the reference."""
    errs = []
    rng = np.random.default_rng(13)
    data = rng.integers(0, 256, 64 * 1024, dtype=np.uint8)

    def worker(t):
        try:
            r = random.Random(t)
            for _ in range(200):
                a = r.randrange(0, 60000)
                L = r.randrange(0, 1519)
                b = data[a:a + L].tobytes()
                if na.ether_fcs(b) != zlib.crc32(b):
                    errs.append((t, a, L))
            out = np.zeros(1000, dtype=np.uint32)
            na.fixed_host(data, 60, 60, 1000, out)
            if not np.array_equal(out, oracle_fixed(oracle, data, 60, 60, 1000)):
                errs.append((t, "batch"))
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errs, errs[:5]


def test_host_calls_keep_the_callers_device(dev, oracle):
    """Host-batch, TX and verify calls make their engine device current only for the call
    (ADVICE r01): the calling thread's current device is unchanged afterwards."""
    before = torch.cuda.current_device()
    host = np.random.default_rng(3).integers(0, 256, 3000 * 1518, dtype=np.uint8)
    out = np.zeros(3000, dtype=np.uint32)
    na.fixed_host(host, 1518, 1518, 3000, out)
    assert torch.cuda.current_device() == before
    ln = np.full(3000, 1514, dtype=np.uint32)
    tx = np.zeros(3000 * 1518, dtype=np.uint8)
    na.tx_host(tx, 1518, ln, 3000)
    assert torch.cuda.current_device() == before
    buf = na.host_buffer(64 * 1518)
    try:
        lens = np.full(64, 1514, dtype=np.uint32)
        na.tx_host(buf, 1518, lens, 64)
        off = np.arange(64, dtype=np.uint64) * 1518
        ok = np.zeros(64, dtype=np.uint8)
        assert na.verify_host(buf, 64 * 1518, off, np.full(64, 1518, dtype=np.uint32), ok, 64) == 0
    finally:
        na.host_free(buf)
    assert torch.cuda.current_device() == before
    assert np.array_equal(out, oracle_fixed(oracle, host, 1518, 1518, 3000))


def test_bad_arguments_are_rejected(dev):
    lib = na.load()
    assert lib.ether_fcs_fixed_dev(None, 1, 1, 1, None, None) == -22
    t = torch.zeros(64, dtype=torch.uint8, device=dev)
    assert lib.ether_fcs_fixed_dev(ctypes.c_void_p(t.data_ptr()), 10, 20, 2, ctypes.c_void_p(t.data_ptr()), None) == -22
    assert lib.ether_fcs_fixed_dev(ctypes.c_void_p(t.data_ptr()), 10, 20, 0, ctypes.c_void_p(t.data_ptr()), None) == 0


hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as hst  # noqa: E402


@settings(max_examples=25, deadline=None, derandomize=True)
@given(hst.lists(hst.tuples(hst.integers(0, 5000), hst.integers(0, 4095)), min_size=1, max_size=300),
       hst.sampled_from(["quarter", "windowed"]))
def test_var_batches_fuzz(dev, batch, kernel):
    """Random lengths (0..5000 B, every segment count up to 4) at random, overlapping offsets with
    every byte alignment, through both variable-length kernels, against zlib.crc32."""
    old = na.set_var_threshold((1 << 63) if kernel == "quarter" else 0)
    try:
        rng = np.random.default_rng(len(batch))
        arena = rng.integers(0, 256, 4096 + 5000 + 64, dtype=np.uint8)
        ln = [L for L, _ in batch]
        off = [o for _, o in batch]
        got = run_var(dev, arena, off, ln)
        for i, (L, o) in enumerate(batch):
            assert got[i] == zlib.crc32(arena[o:o + L].tobytes()), (kernel, L, o)
    finally:
        na.set_var_threshold(old)


# Fixed-length batches above the small-batch threshold with frames of at most 1503 B take the flat
# kernel (len array absent: the length is the batch's) unless a slot kernel takes them (870..1503 B
# with strides whose four frames fit its slot); lengths and strides the route covers.
@pytest.mark.parametrize("L,stride", [(0, 4), (1, 1), (13, 17), (60, 60), (64, 64), (70, 72),
                                      (96, 96), (97, 101), (576, 576), (1000, 1003), (869, 869), (1156, 2100),
                                      (1157, 2100), (1476, 2049), (1490, 1900), (1503, 2100)])
def test_fixed_short_frames_flat_route(dev, oracle, L, stride):
    n = 20000   # > the 16384-frame small-batch threshold
    nbytes = (n - 1) * stride + L + 3
    host = np.random.default_rng(L * 7919 + stride).integers(0, 256, nbytes, dtype=np.uint8)
    base = to_dev(host, dev)
    got = run_fixed(dev, base[3:], stride, L, n)   # odd base alignment
    exp = oracle_fixed(oracle, host[3:].copy(), stride, L, n)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("mode", ["imix", "fixed576"])
def test_flat_kernel_dynamic_windows(dev, oracle, mode):
    """Batches of >= 4 windows (64 frames) per wave take their windows from the work counter:
    1.1 M frames through the flat kernel, every one against the oracle."""
    n = 1100003
    rng = np.random.default_rng(5)
    if mode == "imix":
        ln = rng.choice(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.uint32), n)
        off = np.zeros(n, dtype=np.uint64)
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        total = int(off[-1]) + int(ln[-1])
        arena = rng.integers(0, 256, total + 5, dtype=np.uint8)
        got = run_var(dev, arena, off, ln)
        assert np.array_equal(got, oracle_var(oracle, arena, off, ln))
    else:
        L = 576
        host = rng.integers(0, 256, n * L + 3, dtype=np.uint8)
        d = to_dev(host, dev)
        got = run_fixed(dev, d.data_ptr() + 1, L, L, n)
        assert np.array_equal(got, oracle_fixed(oracle, host[1:], L, L, n))


@pytest.mark.parametrize("L,stride,n,lead", [(2000, 2000, 70001, 1), (1540, 1544, 90003, 0),
                                            (9000, 9000, 40001, 3), (9018, 9024, 33333, 2)])
def test_generic_kernel_dynamic_units(dev, oracle, L, stride, n, lead):
    """Fixed-length batches of >= 4 units (4 frames, one per quarter-wave) per wave of the grid take
    their units from the work counter (guided chunks): every frame against the oracle, twice on
    the same stream (the counter ring's next slot)."""
    host = np.random.default_rng(L + n).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = to_dev(host, dev)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    for _ in range(2):
        got = run_fixed(dev, d.data_ptr() + lead, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))
