"""RX verification: frames carrying their FCS trailer, checked by the CRC residue.

The reference's ether_receive (src/linux/ether.c:180-212) checks no FCS, so there is no
reference output to match. The check is pinned instead to the reference's own TX layout
(src/linux/ether.c:262-263: LE32 of ether_fcs over the covered bytes, right after them) and to
its residue property: ether_fcs(frame || LE32(ether_fcs(frame))) == 0x2144DF1C for every frame
(SURVEY §8c known answers). The expected flag of every frame comes from the oracle's
restatement of src/ether_fcs.c, never from the engine.
"""
import struct

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
RESIDUE = 0x2144DF1C


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    na.load()
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def expected_ok(oracle, arena, off, ln):
    return np.array([int(oracle.oracle_crc32_fast(arena[int(o):].ctypes.data, int(n)) == RESIDUE)
                     for o, n in zip(off, ln)], dtype=np.uint8)


def build_rx_batch(oracle, rng, lens, corrupt_frac=0.2, gap_max=7):
    """Frames laid out as ether_send writes them (covered bytes + LE32 FCS), packed with random
    gaps; a fraction gets one flipped bit (anywhere, trailer included)."""
    total = int(sum(lens)) + gap_max * len(lens) + 64
    arena = rng.integers(0, 256, total, dtype=np.uint8)
    off = np.zeros(len(lens), dtype=np.uint64)
    pos = int(rng.integers(0, 4))
    for i, L in enumerate(lens):
        off[i] = pos
        if L >= 4:
            c = oracle.oracle_ether_fcs(arena[pos:].ctypes.data, L - 4)
            arena[pos + L - 4:pos + L] = np.frombuffer(struct.pack("<I", c), dtype=np.uint8)
        pos += L + int(rng.integers(0, gap_max + 1))
    bad_idx = [i for i in range(len(lens)) if lens[i] > 0 and rng.random() < corrupt_frac]
    for i in bad_idx:
        bit = int(rng.integers(0, 8 * lens[i]))
        arena[int(off[i]) + bit // 8] ^= np.uint8(1 << (bit % 8))
    return arena, off, np.asarray(lens, dtype=np.uint32)


def run_verify_var(dev, arena, off, ln):
    ok = torch.zeros(len(ln), dtype=torch.uint8, device=dev)
    bad = torch.full((1,), 12345, dtype=torch.int64, device=dev)   # must be zeroed by the call
    na.verify_dev(to_dev(arena, dev), arena.nbytes, to_dev(off.view(np.int64), dev),
                  to_dev(ln.view(np.int32), dev), ok, bad, len(ln))
    torch.cuda.synchronize()
    return ok.cpu().numpy(), int(bad.item())


def test_verify_var_all_classes(dev, var_kernel, oracle):
    """Small (<= 96), medium (<= 768), big (> 768) and multi-segment frames, corrupted 20 %."""
    rng = np.random.default_rng(41)
    lens = [int(x) for x in rng.choice([0, 1, 3, 4, 5, 60, 64, 74, 96, 97, 200, 576, 768, 769,
                                        1000, 1518, 1536, 1537, 3000, 9000], 3000)]
    arena, off, ln = build_rx_batch(oracle, rng, lens)
    exp = expected_ok(oracle, arena, off, ln)
    ok, bad = run_verify_var(dev, arena, off, ln)
    assert np.array_equal(ok, exp)
    assert bad == int((exp == 0).sum())
    # frames shorter than 4 bytes can never carry an FCS
    assert not ok[ln < 4].any()


def test_verify_var_edges_and_tiny_arena(dev, var_kernel, oracle):
    """Frames at the very start/end of the arena, and an arena too small for chunk windows."""
    rng = np.random.default_rng(42)
    for lens in ([74], [4, 8, 12], [70, 74, 96], [1514, 74], [5] * 30):
        arena, off, ln = build_rx_batch(oracle, rng, lens, corrupt_frac=0.3, gap_max=0)
        arena = arena[:int(off[-1]) + int(ln[-1])].copy()        # arena ends at the last frame
        exp = expected_ok(oracle, arena, off, ln)
        ok, bad = run_verify_var(dev, arena, off, ln)
        assert np.array_equal(ok, exp), lens
        assert bad == int((exp == 0).sum())


def test_verify_host_matches_device(dev, var_kernel, oracle):
    rng = np.random.default_rng(43)
    lens = [int(x) for x in rng.integers(70, 1519, 20000)]
    arena, off, ln = build_rx_batch(oracle, rng, lens, corrupt_frac=0.05)
    exp = expected_ok(oracle, arena, off, ln)
    ok = np.zeros(len(ln), dtype=np.uint8)
    nbad = na.verify_host(arena, arena.nbytes, off, ln, ok, len(ln))
    assert np.array_equal(ok, exp)
    assert nbad == int((exp == 0).sum())


@pytest.mark.parametrize("n", [1, 5, 64, 65, 300])
def test_verify_host_in_place_small_batches(dev, oracle, n):
    """RX-queue-sized batches in fcs_host_alloc memory take the in-place paths (up to 64 frames of
    up to 1536 B: the small-batch kernel with the frame list in its arguments). Frames of 0..3
    bytes never check, the last frame ends on the allocation's last byte (a page boundary), and
    a fifth of the frames carry a flipped bit."""
    rng = np.random.default_rng(500 + n)
    lens = [int(x) for x in rng.integers(64, 1519, n)]
    lens[:min(n, 4)] = [0, 3, 4, 1536][:min(n, 4)]
    arena, off, ln = build_rx_batch(oracle, rng, lens)
    last = int(off[-1] + ln[-1])
    size = (last + 4095) // 4096 * 4096
    shift = size - last                                # move the frames so the last one ends the buffer
    buf = na.host_buffer(size)
    try:
        buf[:] = 0
        buf[shift:shift + last] = arena[:last]
        off2 = off + np.uint64(shift)
        exp = expected_ok(oracle, buf, off2, ln)
        ok = np.zeros(n, dtype=np.uint8)
        nbad = na.verify_host(buf, size, off2, ln, ok, n)
        assert np.array_equal(ok, exp)
        assert nbad == int((exp == 0).sum())
        assert exp[0] == 0 and (n < 2 or exp[1] == 0)
    finally:
        na.host_free(buf)


@pytest.mark.parametrize("L", [74, 1518, 9018])
def test_verify_fixed_single_and_multi_segment(dev, oracle, L):
    """Fixed stride: the single-segment kernel (<= 1536 B) and the generic multi-segment one."""
    rng = np.random.default_rng(L)
    n = 2000
    lens = [L] * n
    arena, off, ln = build_rx_batch(oracle, rng, lens, corrupt_frac=0.1, gap_max=0)
    base = int(off[0])
    exp = expected_ok(oracle, arena, off, ln)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    d = to_dev(arena, dev)
    na.verify_fixed_dev(d.data_ptr() + base, L, L, n, ok, bad)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), exp)
    assert int(bad.item()) == int((exp == 0).sum())


@pytest.mark.parametrize("L", [64, 576, 869])
def test_verify_fixed_flat_route(dev, oracle, L):
    """Fixed frames of <= 869 B (packed; longer ones take the slot kernels, up to 1503 B with
    strides those do not take) in batches of > 16384 take the flat chunk-stream kernel with no
    length array (p.len == null) and the fused ok/bad epilogue: corrupted frames
    included, ok[] and the bad count against the oracle."""
    rng = np.random.default_rng(L + 1)
    n = 20000
    arena, off, ln = build_rx_batch(oracle, rng, [L] * n, corrupt_frac=0.05, gap_max=0)
    base = int(off[0])
    exp = expected_ok(oracle, arena, off, ln)
    assert 0 < int((exp == 0).sum()) < n
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    d = to_dev(arena, dev)
    na.verify_fixed_dev(d.data_ptr() + base, L, L, n, ok, bad)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), exp)
    assert int(bad.item()) == int((exp == 0).sum())


def test_verify_baseline_size_residue(dev):
    """4 M x 1518-B frames built on the device (FCS of bytes 0..1513 written LE at 1514): all pass;
    then k chosen frames get one bit flipped and exactly those fail (size-independent property)."""
    n, L = 4 << 20, 1518
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, 77, 0)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(arena, L, L - 4, n, crc)
    view = arena.view(n, L)
    view[:, L - 4:] = crc.view(torch.uint8).view(n, 4)          # little-endian, as :263 memcpy
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    na.verify_fixed_dev(arena, L, L, n, ok, bad)
    torch.cuda.synchronize()
    assert int(bad.item()) == 0 and bool(ok.all())
    idx = torch.tensor([0, 1, 12345, n // 2, n - 1], device=dev)
    pos = torch.tensor([0, 1517, 700, 1514, 3], device=dev)
    view[idx, pos] ^= 0x10
    na.verify_fixed_dev(arena, L, L, n, ok, bad)
    torch.cuda.synchronize()
    assert int(bad.item()) == len(idx)
    assert torch.nonzero(ok == 0).flatten().tolist() == sorted(idx.tolist())


def test_verify_counts_every_bad_frame(dev, var_kernel):
    """All-bad batch (random trailers): the per-wave LDS counters must add up to exactly the
    number of frames whose FCS over the whole frame is not the residue (computed by the FCS path)."""
    n, L = 1 << 20, 1518
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, 91, 0)
    crc = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(arena, L, L, n, crc)
    expect = int((crc != RESIDUE).sum().item())
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    na.verify_fixed_dev(arena, L, L, n, ok, bad)
    torch.cuda.synchronize()
    assert int(bad.item()) == expect and int((ok == 0).sum().item()) == expect
    off = torch.arange(n, dtype=torch.int64, device=dev) * L
    ln = torch.full((n,), L, dtype=torch.int32, device=dev)
    na.verify_dev(arena, n * L, off, ln, ok, bad, n)
    torch.cuda.synchronize()
    assert int(bad.item()) == expect
