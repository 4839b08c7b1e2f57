"""GPU parity of the wide LDS-DMA kernel (fcs_wide_kernel<WD>).

Fixed-length frames of 1525..1988 B whose four consecutive frames fit one LDS slot take this kernel
(wide_wd(), fcs_launch.hpp), at one of three window widths:
  - WD 26: 104-B windows every 100 B (cover 1604 B), 7 KiB slots (3 stride + len <= 7150), 13 waves;
    also 1477..1495 B, between the mid-length band (test_gpu_wide_mid.py) and the LDS-DMA kernel
    (front lane 14, lane 15 dropped);
  - WD 30: 120-B windows every 116 B (cover 1860 B), 7 KiB slots, 13 waves: 1605..1787 B at
    stride = len (from 1788 B four frames no longer fit 7 KiB);
  - WD 32: 128-B windows every 124 B (cover 1988 B), 8 KiB slots (3 stride + len <= 8174), 12 waves:
    everything else in the band.
Lane c of a frame reads the window ending step * c before the frame end; every live lane but the
front one masks its first word (its neighbour's last), the front lane cf = (len - 1) / step masks
its leading bytes and starts from INV[zc], the lanes past it are dropped. Every case is checked
bit-exact against the oracle (the CPU restatement of src/ether_fcs.c:4-19): every front-lane
boundary of each width (WD 26: 1600/1601/1604, WD 30: 1624/1625, 1740/1741, WD 32: 124 c + 1 and
124 c + 4), the width switches (1604/1605, 1787/1788) and the band's ends with the lengths just
outside it; strides from no gap to the largest each slot takes (3 stride + len = 7150 and 7151 for
the 7 KiB widths, the largest stride under 8174 for the 8 KiB one); all base alignments, partial
items, the arena-end slot clamp, batches large enough for the dynamic schedule at each width,
verify mode, and a fuzz over the band.
"""
import struct
import zlib

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    na.load()
    return torch.device("cuda:0")


def oracle_fixed(oracle, host: np.ndarray, stride, L, n):
    out = np.empty(n, dtype=np.uint32)
    oracle.oracle_fcs_fixed(host.ctypes.data, stride, L, n, out.ctypes.data, 1, 16)
    return out


def run(dev, d, lead, stride, L, n):
    out = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(d.data_ptr() + lead, stride, L, n, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


# the band's ends and one byte outside; each front lane's first and last lengths (cf = 12 .. 15:
# lengths 124 cf + 1 .. 124 cf + 124, zc = 127 .. 4); the QinQ / baby-giant sizes
LENS = sorted({1476, 1477, 1478, 1480, 1490, 1494, 1495, 1496, 1501, 1524, 1525, 1526, 1530, 1536, 1537, 1548, 1549, 1552, 1600, 1601, 1604, 1605, 1611, 1624, 1625,
               1672, 1673, 1676, 1700, 1740, 1741, 1787, 1788, 1796, 1797, 1800, 1860, 1861, 1864, 1900, 1920,
               1949, 1950, 1984, 1985, 1987, 1988, 1989, 2000})


@pytest.mark.parametrize("L", LENS)
def test_wide_lengths(dev, oracle, L):
    gaps = [0, 1, 3, 8, (8174 - L) // 3 - L]          # the last: the largest stride an 8 KiB slot takes
    s7 = (7150 - L) // 3                               # the largest stride a 7 KiB slot takes ...
    if s7 >= L:                                        # ... (up to 1787 B; from 1788 B none does)
        gaps += [s7 - L, s7 + 1 - L]                   # 3 stride + len <= 7150, and the first stride past it
    for gap in sorted(set(g for g in gaps if g >= 0)):
        stride = L + gap
        for n in (1, 3, 11, 13, 257):
            host = np.random.default_rng(L * 7 + gap * 3 + n).integers(0, 256, n * stride + 16, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            for lead in (0, 1, 2, 3):
                got = run(dev, d, lead, stride, L, n)
                exp = oracle_fixed(oracle, host[lead:], stride, L, n)
                assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L,stride", [(1477, 1477), (1495, 1536), (1525, 1525), (1526, 1536), (1536, 1536), (1560, 1560), (1600, 1600), (1600, 1664),
                                      (1700, 1700), (1787, 1787), (1788, 2000), (1949, 1949), (1988, 1988),
                                      (1988, 2062)])
def test_wide_many_items(dev, oracle, L, stride):
    """More items than the grid's waves (the dynamic schedule) and a second launch reusing the
    counter ring; the last items' slots clamped at the arena end."""
    n = (300 << 20) // stride + 3
    host = np.random.default_rng(L + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[1:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 1, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


@pytest.mark.parametrize("L,stride", [(1552, 1866), (1553, 1866), (1702, 1816), (1703, 1816), (1600, 1850),
                                      (1600, 1851)])
def test_wide_seven_kib_slot_bound(dev, oracle, L, stride):
    """3 stride + len = 7150 is the largest item a 7 KiB slot takes (WD 26 / WD 30); 7151 moves the
    batch to the 128-B windows and 8 KiB slots. Both sides, with enough items for the dynamic
    schedule, at two base alignments."""
    n = (64 << 20) // stride + 5
    host = np.random.default_rng(L * stride).integers(0, 256, n * stride + 16, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    for lead in (0, 3):
        got = run(dev, d, lead, stride, L, n)
        exp = oracle_fixed(oracle, host[lead:], stride, L, n)
        assert np.array_equal(got, exp), (L, stride, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L", [1477, 1490, 1525, 1530, 1536, 1560, 1600, 1700, 1787, 1796, 1922, 1988])
def test_wide_verify_mode(dev, L):
    """RX residue check through the wide kernel: frames of L bytes carrying their FCS, a few
    corrupted; ok[] and the bad count against zlib."""
    n = 4099
    rng = np.random.default_rng(L)
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    for i in range(n):
        f = host[i * L:i * L + L - 4].tobytes()
        host[i * L + L - 4:i * L + L] = np.frombuffer(struct.pack("<I", zlib.crc32(f)), dtype=np.uint8)
    bad_idx = sorted(set(int(x) for x in rng.integers(0, n, 23)) | {0, n - 1})
    for i in bad_idx:
        host[i * L + int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    d = torch.from_numpy(host).to(dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    na.verify_fixed_dev(d, L, L, n, ok, bad)
    torch.cuda.synchronize()
    exp = np.ones(n, dtype=np.uint8)
    exp[bad_idx] = 0
    assert np.array_equal(ok.cpu().numpy(), exp)
    assert int(bad.item()) == len(bad_idx)


hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as hst  # noqa: E402


@settings(max_examples=40, deadline=None, derandomize=True)
@given(hst.integers(1470, 1995), hst.integers(0, 200), hst.integers(1, 2000), hst.integers(0, 15))
def test_wide_fuzz(dev, oracle, L, gap, n, lead):
    """Random lengths across the band and just outside it, gaps, frame counts and base alignments
    against the oracle (the wide kernel where its slot takes the item, the others elsewhere)."""
    stride = L + gap
    host = np.random.default_rng(L ^ (gap << 17) ^ (n << 33) ^ lead).integers(0, 256, n * stride + 32, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = run(dev, d, lead, stride, L, n)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))
