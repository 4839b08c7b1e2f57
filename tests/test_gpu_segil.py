"""GPU parity of the frame-interleaved segment route (fcs_segil_kernel, and fcs_segw_kernel<WD>
where segment_wd() picks wider segments).

Fixed-length frames over 1524 B take the segment route when m = ceil(len / 1524) >= 4, or m = 3 and
len > 3072, or m = 2 and len >= 1950 (fixed_segil(), fcs_launch.hpp),
at any stride: a front segment of len - 1524 (m - 1) bytes, then 1524-B segments; item r of a
wave's unit is segment r of its four frames (one per quarter-wave, four DMA runs), and a frame's
CRC state goes from item to item through lane 15's chain start. Every case is checked bit-exact
against the oracle (the CPU restatement of src/ether_fcs.c:4-19): front segments of 1 to 1524
bytes, both sides of the selection bounds (1949 / 1950, 3072 / 3073 B: the shorter ones keep the
register-load generic kernel; 2285 / 2286 and 3428 / 3429 were round 2's bounds), up to 688 segments (1 MiB), all base alignments, strides with no
gap, odd gaps and large gaps, frame counts that leave partial units, batches large enough for the
dynamic schedule, and verify mode.
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


# front segments of 1 .. 1524 B; the selection bounds (1950, 3073) and one byte below them; round 2's
# bounds (2286 = 0.75 * 3048, 3429 = 0.75 * 4572); the old segmented kernel's bands (2992-3048,
# 8976-9144, 40392-41148)
LENS = [1525, 1530, 1536, 1537, 1949, 1950, 2000, 3072, 3073, 3200, 2285, 2286, 2500, 2992, 3000, 3048, 3049, 3428, 3429, 4572, 4573,
        6000, 6096, 7500, 8976, 9000, 9018, 9143, 9144, 10000, 10472, 16000, 16500, 40392, 41148, 41149,
        64400, 65536, 100000]


@pytest.mark.parametrize("L", LENS)
def test_segil_lengths(dev, oracle, L):
    for gap in (0, 1, 8, 1001):
        stride = L + gap
        for n in ((1, 3, 6, 13, 257) if L < 20000 else (1, 5, 33)):
            host = np.random.default_rng(L * 7 + gap * 3 + n).integers(0, 256, n * stride + 16, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            for lead in (0, 1, 2, 3):
                got = run(dev, d, lead, stride, L, n)
                exp = oracle_fixed(oracle, host[lead:], stride, L, n)
                assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L,stride", [(2500, 2500), (3000, 3000), (3040, 3048), (4500, 4500), (6000, 6001), (7500, 7500),
                                      (9000, 9000), (9000, 9216), (10000, 10003), (16500, 16500), (41148, 41150),
                                      (65536, 65536)])
def test_segil_many_units(dev, oracle, L, stride):
    """More units than the grid's waves (every wave walks several units; the dynamic schedule for
    the larger batches), and a second launch reusing the counter ring."""
    n = max(40001, (300 << 20) // stride) if L < 10000 else 20001
    host = np.random.default_rng(L + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[3:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 3, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


@pytest.mark.parametrize("L", [2500, 3000, 4500, 6000, 7500, 9000, 9022, 10000, 16500, 41148, 65536])
def test_segil_verify_mode(dev, L):
    """RX residue check through the interleaved segment kernel: frames of L bytes carrying their FCS, a few
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
@given(hst.integers(1525, 70000), hst.integers(0, 3000), hst.integers(1, 600), hst.integers(0, 15))
def test_segil_fuzz(dev, oracle, L, gap, n, lead):
    """Random fixed lengths over 1524 B (either kernel, by the selection bound), gaps, frame counts
    and base alignments against the oracle."""
    stride = L + gap
    host = np.random.default_rng(L ^ (gap << 17) ^ (n << 33) ^ lead).integers(0, 256, n * stride + 32, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = run(dev, d, lead, stride, L, n)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))
