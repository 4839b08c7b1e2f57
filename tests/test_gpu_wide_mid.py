"""GPU parity of the mid-length wide kernels (fcs_wide_kernel<WD>, WD = 15 .. 24).

Fixed-length frames of 870..1476 B whose four consecutive frames fit a 6 KiB slot take the narrowest
bank-safe window width whose 16 windows cover the frame (fcs_launch.hpp wide_mid_wd: WD - 1 not a
multiple of 4, so WD 17 and 21 are skipped): windows of 4 WD bytes every 4 WD - 4 bytes, 16 waves.
Before round 4 these lengths took the flat chunk stream, which keeps the shorter ones. Every case is
checked bit-exact against the oracle (the CPU restatement of src/ether_fcs.c:4-19): both ends of
every width's band, the band's own ends and the lengths just outside it (869 / 870, 1476 / 1477),
strides from no gap to the largest
a 6 KiB slot takes (3 stride + len = 6126) and one past it, all base alignments, partial items, the
arena-end slot clamp, batches large enough for the dynamic schedule, verify mode, and a fuzz over
the band. The CPU model of the same decomposition: tests/test_kernel_model.py::test_wide_kernel_model.
"""
import struct
import zlib

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

WIDTHS = [wd for wd in range(15, 25) if (wd - 1) % 4]


def cover(wd):
    return 15 * (4 * wd - 4) + 4 * wd


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


# each width's narrowest and widest frame, and the band's ends with the lengths just outside
LENS = sorted({700, 837, 869, 870, 1000, 1156, 1157, 1476, 1477, 1500} | {cover(wd) for wd in WIDTHS} |
              {cover(prev) + 1 for prev, wd in zip(WIDTHS[:-1], WIDTHS[1:])})


@pytest.mark.parametrize("L", LENS)
def test_mid_lengths(dev, oracle, L):
    s6 = (6126 - L) // 3   # the largest stride a 6 KiB slot takes
    gaps = sorted(g for g in {0, 1, 3, 8, s6 - L, s6 + 1 - L} if g >= 0)
    for gap in gaps:
        stride = L + gap
        for n in (1, 3, 13, 257):
            host = np.random.default_rng(L * 7 + gap * 3 + n).integers(0, 256, n * stride + 16, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            for lead in (0, 1, 2, 3):
                got = run(dev, d, lead, stride, L, n)
                exp = oracle_fixed(oracle, host[lead:], stride, L, n)
                assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L,stride", [(870, 870), (900, 964), (1000, 1000), (1092, 1092), (1157, 1157), (1200, 1200), (1220, 1300), (1221, 1221),
                                      (1300, 1300), (1400, 1400), (1476, 1476), (1476, 1550)])
def test_mid_many_items(dev, oracle, L, stride):
    """More items than the grid's waves (the dynamic schedule) and a second launch reusing the
    counter ring; the last items' slots clamped at the arena end."""
    n = (200 << 20) // stride + 3
    host = np.random.default_rng(L + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[1:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 1, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


@pytest.mark.parametrize("L", [870, 900, 964, 965, 1093, 1157, 1220, 1221, 1349, 1412, 1413, 1476])
def test_mid_verify_mode(dev, L):
    """RX residue check through the mid-length kernels: frames of L bytes carrying their FCS, a few
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
@given(hst.integers(800, 1500), hst.integers(0, 400), hst.integers(1, 3000), hst.integers(0, 15))
def test_mid_fuzz(dev, oracle, L, gap, n, lead):
    """Random lengths across the band and just outside it, gaps, frame counts and base alignments
    against the oracle (the mid-length kernels where a 6 KiB slot takes the item, others elsewhere)."""
    stride = L + gap
    host = np.random.default_rng(L ^ (gap << 17) ^ (n << 33) ^ lead).integers(0, 256, n * stride + 32, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = run(dev, d, lead, stride, L, n)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))
