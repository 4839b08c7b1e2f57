"""GPU parity of the short-frame kernel (fcs_short_kernel<W>).

Fixed-length batches of more than 16384 frames of 1..128 B take one lane per frame (fcs_launch.hpp
fixed_short / short_wd): the W-dword window ending at the frame end (W = 16 up to 64 B, 24 up to
96 B, 32 up to 128 B) in registers, the zc = 4 W - len bytes before the frame start masked, two
chains from INV[zc] merged with A_{2 W}. Every case is checked bit-exact against the oracle (the CPU
restatement of src/ether_fcs.c:4-19): every window width's shortest and longest frame and the
lengths just outside the kernel (129 B takes the flat kernel), the minimum Ethernet sizes (60/64 B,
and 70/74 B, the smallest frame ether_send builds, src/linux/ether.c:222-224), strides from packed
to 1518, all base alignments (a first frame whose window reaches before the arena start takes the
guarded loads), batch sizes just over the threshold and large enough for the dynamic schedule,
verify mode, and a fuzz.
"""
import struct
import zlib

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N_MIN = 16385   # one more than the small-batch threshold (fcs_engine_set_var_threshold default)


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


LENS = [1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 32, 33, 47, 48, 59, 60, 61, 63, 64, 65, 70, 74, 78, 80, 95, 96,
        97, 100, 127, 128, 129]


@pytest.mark.parametrize("L", LENS)
def test_short_lengths_strides_alignments(dev, oracle, L):
    for stride in sorted({L, L + 1, L + 3, 64, 96, 128, 200} - {s for s in range(L)}):
        n = N_MIN + (L % 7)
        host = np.random.default_rng(L * 131 + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
        d = torch.from_numpy(host).to(dev)
        for lead in (0, 1, 2, 3):
            got = run(dev, d, lead, stride, L, n)
            exp = oracle_fixed(oracle, host[lead:], stride, L, n)
            assert np.array_equal(got, exp), (L, stride, lead, int(np.argmax(got != exp)))


@pytest.mark.parametrize("L,stride", [(60, 60), (64, 64), (74, 74), (96, 96), (128, 128), (64, 1518)])
def test_short_many_items(dev, oracle, L, stride):
    """More items than the grid's waves (the dynamic schedule) and a second launch reusing the
    counter ring; odd base."""
    n = (1 << 20) + 7 if stride < 1000 else 200003
    host = np.random.default_rng(L + stride).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[3:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 3, stride, L, n)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


def test_short_known_answers(dev):
    """Zero and 0xFF frames of 60 B against the reference's known answers."""
    n = N_MIN
    for fill, want in ((0x00, 0x04128908), (0xFF, 0xF48CF14D)):
        d = torch.full((n * 60,), fill, dtype=torch.uint8, device=dev)
        got = run(dev, d, 0, 60, 60, n)
        assert (got == want).all(), (hex(fill), hex(int(got[0])))


@pytest.mark.parametrize("L", [5, 60, 64, 74, 100, 128])
def test_short_verify_mode(dev, L):
    """RX residue check through the short-frame kernel: frames of L bytes carrying their FCS, a few
    corrupted; ok[] and the bad count against zlib."""
    n = N_MIN + 11
    rng = np.random.default_rng(L)
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    for i in range(n):
        f = host[i * L:i * L + L - 4].tobytes()
        host[i * L + L - 4:i * L + L] = np.frombuffer(struct.pack("<I", zlib.crc32(f)), dtype=np.uint8)
    bad_idx = sorted(set(int(x) for x in rng.integers(0, n, 29)) | {0, n - 1})
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
@given(hst.integers(1, 140), hst.integers(0, 300), hst.integers(N_MIN, 40000), hst.integers(0, 15))
def test_short_fuzz(dev, oracle, L, gap, n, lead):
    """Random lengths across the kernel and just past it, gaps, frame counts and base alignments."""
    stride = L + gap
    host = np.random.default_rng(L ^ (gap << 17) ^ (n << 33) ^ lead).integers(0, 256, n * stride + 32, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    got = run(dev, d, lead, stride, L, n)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))
