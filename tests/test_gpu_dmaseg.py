"""GPU parity of the segmented LDS-DMA kernel (fcs_dmaseg_kernel).

Fixed-length frames over 1524 B that split into m = ceil(len / 1524) <= 27 segments of
Ls = floor(len / m) >= 1496 bytes (front segment Ls + len mod m <= 1524) and are packed
(stride - len <= 8) take this kernel: four consecutive segments of the stream per wave item, each
placed in its frame by A_{Ls s} (place tables for s >= 5 composed at staging), the frame's partial
XOR carried from item to item. Every case is checked bit-exact against the oracle (the CPU
restatement of src/ether_fcs.c:4-19): both ends of the bands of m = 2..6, 11, 13 and 27, all base
alignments, strides with and without gaps, frame counts that leave partial units and partial items,
batches large enough for the dynamic schedule, and verify mode. Lengths outside the bands or over 27
segments (1530, 2000, 9143, 10000, 16000, 41149, 65536, ...) take the register-load kernels and are
checked the same way.
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


# bands [1496 m, 1524 m]: m = 2 .. 6 (6: jumbo), 7, 11, 13, 27 (this kernel), 43 (over the segment
# limit); lengths outside every band
LENS = [2992, 2993, 3000, 3047, 3048, 4488, 4500, 4572, 5984, 6000, 6096, 7480, 7500, 8976, 9000,
        9018, 9142, 9144, 10472, 16500, 19448, 19812, 40392, 41148, 64400, 1530, 2000, 9143, 10000,
        16000, 41149, 65536]


@pytest.mark.parametrize("L", LENS)
def test_dmaseg_lengths(dev, oracle, L):
    for gap in (0, 1, 8):
        stride = L + gap
        for n in (1, 3, 6, 13, 257):
            host = np.random.default_rng(L * 7 + gap * 3 + n).integers(0, 256, n * stride + 16, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            for lead in (0, 1, 2, 3):
                got = run(dev, d, lead, stride, L, n)
                exp = oracle_fixed(oracle, host[lead:], stride, L, n)
                assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L,stride", [(3000, 3000), (3040, 3048), (4500, 4500), (6000, 6001), (7500, 7500), (9000, 9000),
                                      (16500, 16500), (41148, 41150)])
def test_dmaseg_many_units(dev, oracle, L, stride):
    """More units than the grid's waves (every wave walks several units; the dynamic schedule for
    the larger batches), and a second launch reusing the counter ring."""
    n = max(40001, (300 << 20) // stride) if L < 10000 else 20001
    host = np.random.default_rng(L + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[3:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 3, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


@pytest.mark.parametrize("L", [3000, 4500, 6000, 7500, 9000, 9022, 16500, 41148])
def test_dmaseg_verify_mode(dev, L):
    """RX residue check through the segmented kernel: frames of L bytes carrying their FCS, a few
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
