"""GPU parity of the windowed variable-length path on packed and unpacked arenas.

Windowed batches (more than 16384 frames, and short fixed lengths) take fcs_flat_kernel. The
span-DMA variant measured in round 2 (removed) staged each item's 64 chunks
through LDS as one contiguous span when the item's frames were packed and fell back to register
loads per item when they were not (gaps, offsets out of order, a frame over 1536 B between
two others); these tests aim at both sides of that choice and at the span's edges (first frame at
the arena start, last frame at the arena end, empty and 1-byte frames, frames of exactly k x 96
bytes, which make the longest spans) and run against either build (NSTACK_FCS_LIB selects the
library). Every frame is checked bit-exact against the oracle's restatement of
src/ether_fcs.c:4-19.
"""
import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N = 20000   # > the 16384-frame small-batch threshold: the windowed (span) kernel


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    na.load()
    return torch.device("cuda:0")


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def oracle_var(oracle, arena, off, ln):
    out = np.empty(len(off), dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    oracle.oracle_fcs_batch(arena.ctypes.data, off.ctypes.data, ln.ctypes.data, out.ctypes.data, len(off), 1)
    return out


def run_var(dev, arena, off, ln, arena_bytes=None, base=0):
    """The batch through the engine. off: offsets into the numpy arena; the engine is handed the
    arena from byte `base` on (arena_bytes long) and offsets relative to it."""
    t = to_dev(arena, dev)
    o = to_dev((np.asarray(off, dtype=np.uint64) - np.uint64(base)).view(np.int64), dev)
    l_ = to_dev(np.asarray(ln, dtype=np.uint32).view(np.int32), dev)
    out = torch.empty(len(off), dtype=torch.int32, device=dev)
    nb = arena.nbytes - base if arena_bytes is None else arena_bytes
    na.batch_dev(t.data_ptr() + base, nb, o, l_, out, len(off))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def packed(ln, lead=0, tail=0, seed=0):
    ln = np.asarray(ln, dtype=np.uint32)
    off = np.zeros(len(ln), dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    off += lead
    total = lead + int(ln.sum(dtype=np.uint64)) + tail
    arena = np.random.default_rng(seed).integers(0, 256, max(total, 1), dtype=np.uint8)
    return arena, off, ln


@pytest.mark.parametrize("lead,tail", [(0, 0), (1, 3), (7, 0), (0, 13), (100, 200)])
def test_packed_imix_edges(dev, oracle, lead, tail):
    """Packed IMIX; the first frame at (or just after) the arena start, the last at its end."""
    rng = np.random.default_rng(lead * 31 + tail)
    ln = rng.choice(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.uint32), N)
    arena, off, ln = packed(ln, lead, tail, seed=lead + tail)
    got = run_var(dev, arena, off, ln, arena_bytes=arena.nbytes - lead, base=lead)
    exp = oracle_var(oracle, arena, off, ln)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("L", [96, 192, 960, 1536])
def test_packed_multiples_of_96(dev, oracle, L):
    """Frames of k x 96 bytes: no overlap between frames' chunks, items span a full 6 KiB (and,
    from a misaligned start, 6 KiB + 15 B: those items take the register loads)."""
    for lead in (0, 5, 12):
        arena, off, ln = packed(np.full(N, L, dtype=np.uint32), lead, 0, seed=L + lead)
        got = run_var(dev, arena, off, ln, arena_bytes=arena.nbytes - lead, base=lead)
        assert np.array_equal(got, oracle_var(oracle, arena, off, ln)), lead


def test_packed_with_empty_short_and_long_frames(dev, oracle):
    """Empty, 1..4-byte and 1537..9000-byte frames in a packed stream (windows with frames over
    1536 B are not dense: chunk ranks go through the frame list, the long frames through the
    segment loop, and the items across them through register loads)."""
    rng = np.random.default_rng(11)
    pool = np.array([0, 1, 2, 3, 4, 64, 95, 97, 576, 1518, 1536, 1537, 2000, 9000], dtype=np.uint32)
    ln = rng.choice(pool, N, p=[.03, .03, .03, .03, .03, .3, .05, .05, .2, .15, .04, .02, .02, .02])
    arena, off, ln = packed(ln, 3, 5, seed=12)
    got = run_var(dev, arena, off, ln, arena_bytes=arena.nbytes - 3, base=3)
    assert np.array_equal(got, oracle_var(oracle, arena, off, ln))


@pytest.mark.parametrize("gap", [1, 8, 40, 200])
def test_gaps_between_frames(dev, oracle, gap):
    """Gaps widen an item's span past the slot for some items: those load into registers."""
    rng = np.random.default_rng(gap)
    ln = rng.choice(np.array([64, 128, 576, 1000, 1518], dtype=np.uint32), N)
    gaps = rng.integers(0, gap + 1, N).astype(np.uint64)
    off = np.zeros(N, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1].astype(np.uint64) + gaps[:-1])
    arena = rng.integers(0, 256, int(off[-1]) + int(ln[-1]) + 16, dtype=np.uint8)
    assert np.array_equal(run_var(dev, arena, off, ln), oracle_var(oracle, arena, off, ln))


def test_offsets_out_of_order_and_overlapping(dev, oracle):
    """Frames listed in a shuffled order and frames sharing bytes (a frame inside another)."""
    rng = np.random.default_rng(5)
    ln = rng.choice(np.array([64, 576, 1518], dtype=np.uint32), N)
    arena, off, ln = packed(ln, 0, 0, seed=6)
    perm = rng.permutation(N)
    off2, ln2 = off[perm].copy(), ln[perm].copy()
    # every 7th frame: a sub-frame of its own bytes, shifted in by a few bytes
    sub = np.arange(0, N, 7)
    cut = np.minimum(ln2[sub], rng.integers(0, 9, len(sub)).astype(np.uint32))
    off2[sub] += cut
    ln2[sub] -= cut
    assert np.array_equal(run_var(dev, arena, off2, ln2), oracle_var(oracle, arena, off2, ln2))


@pytest.mark.parametrize("L", [64, 100, 576, 1000, 1503])
def test_fixed_short_route_packed_and_strided(dev, oracle, L):
    """Short fixed lengths take the same kernel without a length array (len == null)."""
    for stride, lead in ((L, 0), (L, 9), (L + 4, 2), (2 * L, 0)):
        n = N
        host = np.random.default_rng(L + stride + lead).integers(0, 256, lead + n * stride + 8, dtype=np.uint8)
        t = to_dev(host, dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        na.fixed_dev(t.data_ptr() + lead, stride, L, n, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        off = np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(lead)
        exp = oracle_var(oracle, host, off, np.full(n, L, dtype=np.uint32))
        assert np.array_equal(got, exp), (stride, lead)


def test_verify_mode_packed(dev, oracle):
    """RX verify through the span kernel: packed frames with their FCS trailer, some corrupted."""
    import struct
    rng = np.random.default_rng(21)
    ln = rng.choice(np.array([68, 580, 1522], dtype=np.uint32), N)
    arena, off, ln = packed(ln, 0, 0, seed=22)
    for o, L in zip(off, ln):
        c = oracle.oracle_ether_fcs(arena[int(o):].ctypes.data, int(L) - 4)
        arena[int(o) + L - 4:int(o) + L] = np.frombuffer(struct.pack("<I", c), dtype=np.uint8)
    bad_idx = rng.choice(N, N // 10, replace=False)
    for i in bad_idx:
        arena[int(off[i]) + int(rng.integers(0, ln[i]))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    exp = np.array([int(oracle.oracle_crc32_fast(arena[int(o):].ctypes.data, int(L)) == 0x2144DF1C)
                    for o, L in zip(off, ln)], dtype=np.uint8)
    t = to_dev(arena, dev)
    ok = torch.empty(N, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    na.verify_dev(t, arena.nbytes, to_dev(off.view(np.int64), dev), to_dev(ln.view(np.int32), dev), ok, bad, N)
    torch.cuda.synchronize()
    assert np.array_equal(ok.cpu().numpy(), exp)
    assert int(bad.item()) == int((exp == 0).sum())


def test_large_packed_imix_dynamic(dev, oracle):
    """2.2 M packed IMIX frames (dynamic windows, many waves' spans at once); every frame checked."""
    rng = np.random.default_rng(99)
    n = 2200001
    ln = rng.choice(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.uint32), n)
    arena, off, ln = packed(ln, 0, 0, seed=98)
    assert np.array_equal(run_var(dev, arena, off, ln), oracle_var(oracle, arena, off, ln))
