"""GPU parity of the arena-stream kernel (fcs_stream_kernel) and of its hand-off
to fcs_flat_kernel for the units it does not take.

Windowed variable-length batches (more than 16384 frames, with offsets) go through the stream
kernel unit by unit (512 frames): units whose frames are packed and 64..1536 B long are computed
there, every other unit is listed for fcs_flat_kernel. Every frame is checked bit-exact against the
oracle's restatement of src/ether_fcs.c:4-19, and fcs_debug_stream_listed() shows which path took
the units, so a silent hand-off of everything to the flat kernel cannot pass as stream coverage.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import nstack_amd as na  # noqa: E402

pytestmark = pytest.mark.gpu

UNIT = 512   # frames per unit of the product build (checked against the library below)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    global UNIT
    UNIT = na.stream_unit_frames()   # measurement builds may use other unit sizes
    return torch.device("cuda:0")


def _run(dev, oracle, host, off, ln, verify=False):
    n = len(ln)
    d = torch.from_numpy(host).to(dev)
    o = torch.from_numpy(off.astype(np.uint64).view(np.int64)).to(dev)
    l_ = torch.from_numpy(ln.astype(np.uint32).view(np.int32)).to(dev)
    out = torch.full((n,), 0x5A5A5A5A, dtype=torch.int32, device=dev)
    na.batch_dev(d, host.size, o, l_, out, n)
    got = out.cpu().numpy().view(np.uint32)
    exp = np.zeros(n, dtype=np.uint32)
    offc = np.ascontiguousarray(off, dtype=np.uint64)
    lnc = np.ascontiguousarray(ln, dtype=np.uint32)
    oracle.oracle_fcs_batch(host.ctypes.data, offc.ctypes.data, lnc.ctypes.data, exp.ctypes.data, n, 8)
    listed = na.stream_listed()
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} frames differ, first {int(bad[0])} (len {int(ln[bad[0]])})"
    return listed


def _packed(lens, base, seed, tail=64):
    lens = np.asarray(lens, dtype=np.uint64)
    off = base + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    total = int(off[-1] + lens[-1]) + tail
    host = np.random.default_rng(seed).integers(0, 256, total, dtype=np.uint8)
    return host, off, lens.astype(np.uint32)


def _imix(n, seed):
    return np.random.default_rng(seed).choice(np.array([64, 576, 1518], dtype=np.uint32), n, p=[7 / 12, 4 / 12, 1 / 12])


@pytest.mark.parametrize("base", [0, 1, 2, 3, 5, 16, 63, 4095])
def test_imix_packed_all_units_streamed(dev, oracle, base):
    n = 40000 + base
    host, off, ln = _packed(_imix(n, base), base, base)
    assert _run(dev, oracle, host, off, ln) == 0


@pytest.mark.parametrize("L", [64, 65, 127, 128, 576, 1000, 1518, 1535, 1536])
def test_fixed_lengths_packed(dev, oracle, L):
    n = 20000 + 3
    host, off, ln = _packed(np.full(n, L), 7, L)
    assert _run(dev, oracle, host, off, ln) == 0


def test_random_lengths_packed(dev, oracle):
    ln = np.random.default_rng(3).integers(64, 1537, 60000)
    host, off, ln = _packed(ln, 9, 3)
    assert _run(dev, oracle, host, off, ln) == 0


def test_units_ending_on_item_boundaries(dev, oracle):
    """512 frames of 64 B from a 16-B aligned start fill exactly 8 items: every unit's last frame
    ends at the end of its last item (the close without an end mark)."""
    n = 64 * UNIT + 100
    host, off, ln = _packed(np.full(n, 64), 0, 11)
    assert _run(dev, oracle, host, off, ln) == 0
    host, off, ln = _packed(np.full(n, 1024), 32, 12)   # 4 frames per item, ends on item edges
    assert _run(dev, oracle, host, off, ln) == 0


def test_mixed_units_hand_off(dev, oracle):
    """Units broken in different ways are listed for fcs_flat_kernel; the others stream. Breaks:
    a 63-B frame, a 1537-B frame, an empty frame, a gap, two frames swapped, overlapping frames."""
    n = 40 * max(UNIT, 512)   # above the windowed-path threshold (16384 frames) for any unit size
    ln = _imix(n, 21).astype(np.uint64)
    breaks = {3: "short", 7: "long", 11: "empty", 17: "gap", 23: "swap", 29: "overlap"}
    ln[3 * UNIT + 100] = 63
    ln[7 * UNIT + 5] = 1537
    ln[11 * UNIT + 511] = 0
    off = 13 + np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    off[17 * UNIT + 200:] += 40                               # a gap inside unit 17
    a, b = 23 * UNIT + 7, 23 * UNIT + 8                        # swapped order inside unit 23
    off[a], off[b] = off[b], off[a]
    ln[a], ln[b] = ln[b], ln[a]
    off[29 * UNIT + 300] -= 8                                  # overlaps its predecessor
    total = int((off + ln).max()) + 64
    host = np.random.default_rng(21).integers(0, 256, total, dtype=np.uint8)
    listed = _run(dev, oracle, host, off, ln.astype(np.uint32))
    assert listed == len(breaks) + 0, listed


def test_unit_boundaries_between_streamed_units_need_not_touch(dev, oracle):
    """Units are independent: consecutive units may be separated by gaps or out of order."""
    U = 40 * max(UNIT, 512) // UNIT   # above the windowed-path threshold for any unit size
    n = U * UNIT
    ln = _imix(n, 31).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    order = np.random.default_rng(5).permutation(U)           # units stored out of order, with gaps
    blocks = [(off[u * UNIT:(u + 1) * UNIT] - off[u * UNIT], ln[u * UNIT:(u + 1) * UNIT]) for u in range(U)]
    pos = 7
    place = {}
    for u in order:
        place[u] = pos
        pos += int(blocks[u][0][-1] + blocks[u][1][-1]) + 33 + int(u)
    off2 = np.concatenate([blocks[u][0] + place[u] for u in range(U)]).astype(np.uint64)
    host = np.random.default_rng(31).integers(0, 256, pos + 64, dtype=np.uint8)
    assert _run(dev, oracle, host, off2, ln.astype(np.uint32)) == 0


def test_all_units_handed_off(dev, oracle):
    """A TX-slot arena (1536-B slots, 1514-B frames: gaps) streams nothing; the flat kernel takes all."""
    n = 20000
    off = (np.arange(n, dtype=np.uint64) * 1536 + 3).astype(np.uint64)
    ln = np.full(n, 1514, dtype=np.uint32)
    host = np.random.default_rng(4).integers(0, 256, n * 1536 + 64, dtype=np.uint8)
    listed = _run(dev, oracle, host, off, ln)
    assert listed == (n + UNIT - 1) // UNIT


def test_partial_last_unit_and_arena_edges(dev, oracle):
    """The batch fills the arena exactly (first frame at its start, last frame at its end), and
    the last unit holds fewer than 512 frames."""
    n = 3 * UNIT + 77 + 16384
    ln = _imix(n, 41)
    host, off, ln = _packed(ln, 0, 41, tail=0)
    assert _run(dev, oracle, host, off, ln) == 0


def test_verify_mode_through_stream(dev, oracle):
    """RX verification (residue check) on a packed IMIX batch with trailers, some corrupted."""
    import zlib
    n = 30000
    ln = _imix(n, 51)
    host, off, ln = _packed(ln, 5, 51)
    # give every frame a valid trailer: the last 4 bytes are the LE FCS of the bytes before them
    for i in range(n):
        o, L = int(off[i]), int(ln[i])
        host[o + L - 4:o + L] = np.frombuffer(zlib.crc32(host[o:o + L - 4].tobytes()).to_bytes(4, "little"), np.uint8)
    bad_idx = [0, 511, 512, 9999, n - 1]
    for i in bad_idx:
        host[int(off[i]) + 1] ^= 0x40
    d = torch.from_numpy(host).to(dev)
    o = torch.from_numpy(off.astype(np.uint64).view(np.int64)).to(dev)
    l_ = torch.from_numpy(ln.astype(np.int32)).to(dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    badc = torch.zeros(1, dtype=torch.int64, device=dev)
    na.verify_dev(d, host.size, o, l_, ok, badc, n)
    assert int(badc.item()) == len(bad_idx)
    okh = ok.cpu().numpy()
    assert sorted(np.nonzero(okh == 0)[0].tolist()) == bad_idx
    assert na.stream_listed() == 0


hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as hst  # noqa: E402

_KINDS = ["imix", "random", "fixed", "short", "long", "empty", "gap", "swap", "overlap", "jumbo"]


@settings(max_examples=12, deadline=None, derandomize=True)
@given(kinds=hst.lists(hst.sampled_from(_KINDS), min_size=34, max_size=48),
       base=hst.integers(0, 4095), shuffle=hst.booleans(), seed=hst.integers(0, 2**31 - 1))
def test_unit_mix_fuzz(dev, oracle, kinds, base, shuffle, seed):
    """Random unit compositions above the windowed threshold: packed units of IMIX, random or fixed
    lengths stream; units broken one way (a 63-B, 1537-B or empty frame, a gap, a swap, an overlap)
    or made of jumbo frames are handed to fcs_flat_kernel. Units may be stored out of order with gaps
    between them. Every frame against the oracle, and the hand-off count against the broken units."""
    rng = np.random.default_rng(seed)
    U = len(kinds)
    lens, rel, broken = [], [], 0
    for k in kinds:
        if k == "fixed":
            ln = np.full(UNIT, int(rng.integers(64, 1537)), dtype=np.int64)
        elif k == "random":
            ln = rng.integers(64, 1537, UNIT)
        elif k == "jumbo":
            ln = rng.integers(1537, 9019, UNIT)
        else:
            ln = _imix(UNIT, int(rng.integers(1 << 30))).astype(np.int64)
        ln = ln.astype(np.int64)
        i = int(rng.integers(0, UNIT - 1))
        if k == "short":
            ln[i] = int(rng.integers(1, 64))
        elif k == "long":
            ln[i] = int(rng.integers(1537, 3000))
        elif k == "empty":
            ln[i] = 0
        o = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.int64)
        if k == "gap":
            o[i + 1:] += int(rng.integers(1, 70))
        elif k == "swap":
            o[i], o[i + 1] = o[i + 1], o[i]
            ln[i], ln[i + 1] = ln[i + 1], ln[i]
        elif k == "overlap":
            o[i + 1] -= int(rng.integers(1, 16))
        broken += k in ("short", "long", "empty", "gap", "swap", "overlap", "jumbo")
        lens.append(ln)
        rel.append(o)
    order = rng.permutation(U) if shuffle else np.arange(U)
    place, pos = {}, base
    for u in order:
        place[u] = pos
        pos += int((rel[u] + lens[u]).max()) + int(rng.integers(0, 40))
    off = np.concatenate([rel[u] + place[u] for u in range(U)]).astype(np.uint64)
    ln = np.concatenate(lens).astype(np.uint32)
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    listed = _run(dev, oracle, host, off, ln)
    assert listed == broken, (listed, broken)
