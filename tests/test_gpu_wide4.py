"""GPU parity of the four-lane wide kernels (fcs_wide_kernel<WD, 4>, WD = 9 .. 26 but 17).

Fixed-length frames of 130..399 B whose sixteen consecutive frames fit the width's slot (6 KiB up to
WD 24, 7 KiB above) take four lanes per frame and sixteen frames per wave item: the narrowest width
whose four windows (4 WD bytes every 4 WD - 4 bytes) cover the frame, unless the frames of a
32-lane half pile onto a bank (wide_bank_load > 2: those keep the flat kernel). Every case is checked
bit-exact against the oracle (the CPU restatement of src/ether_fcs.c:4-19): both ends of every
width's band, the band's own ends and the lengths just outside it (129 / 130, 399 / 400), strides
from no gap to the largest the slot takes and one past it, all base alignments, partial items, the
arena-end slot clamp, batches large enough for the dynamic schedule, verify mode, and a fuzz.
"""
import struct
import zlib

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

WIDTHS = [wd for wd in range(9, 27) if (wd - 1) % 16]


def cover(wd):
    return 3 * (4 * wd - 4) + 4 * wd


def slot(wd):
    return 7168 if wd > 24 else 6144


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


LENS = sorted({128, 129, 130, 131, 150, 192, 200, 256, 300, 320, 333, 384, 380, 399, 400} | {cover(wd) for wd in WIDTHS if cover(wd) >= 130} |
              {cover(wd) + 1 for wd in WIDTHS if 130 <= cover(wd) < 399})


@pytest.mark.parametrize("L", LENS)
def test_wide4_lengths(dev, oracle, L):
    wd = next((w for w in WIDTHS if cover(w) >= L), 26)
    smax = (slot(wd) - 18 - L) // 15   # the largest stride the width's slot takes
    gaps = sorted(g for g in {0, 1, 3, 8, smax - L, smax + 1 - L} if g >= 0)
    for gap in gaps:
        stride = L + gap
        for n in (1, 15, 17, 33, 257):
            host = np.random.default_rng(L * 7 + gap * 3 + n).integers(0, 256, n * stride + 16, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            for lead in (0, 1, 2, 3):
                got = run(dev, d, lead, stride, L, n)
                exp = oracle_fixed(oracle, host[lead:], stride, L, n)
                assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L,stride", [(130, 130), (150, 150), (200, 200), (256, 256), (300, 300), (320, 320),
                                      (333, 333), (372, 372), (384, 384), (399, 399), (399, 440)])
def test_wide4_many_items(dev, oracle, L, stride):
    """More items than the grid's waves (the dynamic schedule) and a second launch reusing the
    counter ring; the last items' slots clamped at the arena end."""
    n = (200 << 20) // stride + 5
    host = np.random.default_rng(L + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[1:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 1, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


@pytest.mark.parametrize("L", [130, 148, 149, 200, 244, 245, 300, 399])
def test_wide4_verify_mode(dev, L):
    """RX residue check through the four-lane kernels: frames of L bytes carrying their FCS, a few
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
@given(hst.integers(120, 420), hst.integers(0, 200), hst.integers(1, 3000), hst.integers(0, 15))
def test_wide4_fuzz(dev, oracle, L, gap, n, lead):
    """Random lengths across the band and just outside it, gaps, frame counts and base alignments."""
    stride = L + gap
    host = np.random.default_rng(L ^ (gap << 17) ^ (n << 33) ^ lead).integers(0, 256, n * stride + 32, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = run(dev, d, lead, stride, L, n)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))
