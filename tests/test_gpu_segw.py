"""GPU parity of the wide-window segment kernel (fcs_segw_kernel<WD>).

Fixed lengths the segment route takes (fixed_segil(), fcs_launch.hpp) run in segments of the wide
kernel's cover when segment_wd() finds that cheaper than 1524-B segments: WD 15..23 windows
(900..1412-B segments) or 26 / 30 / 32 (1604 / 1860 / 1988 B). The front segment of L - C (m - 1)
bytes carries the wide kernel's front lane (cf, zc), the other segments carry the frame's CRC state into lane 15. Every case is
bit-exact against the oracle (the CPU restatement of src/ether_fcs.c:4-19). The lengths are picked
through the product's own route (fcs_debug_fixed_route), so the test follows segment_wd()'s cost
constant: front segments at every front-lane edge (1..5 bytes, around each multiple of the window
step, the whole cover), 2..8 segments, and the launched kernel is checked to be the routed one.
"""
import struct
import zlib

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

WIDTHS = [15, 16, 18, 19, 20, 22, 23, 26, 30, 32]   # fcs_launch.hpp segment_wd candidates besides 24
STEP = {wd: 4 * wd - 4 for wd in WIDTHS}
COVER = {wd: 15 * STEP[wd] + 4 * wd for wd in WIDTHS}
BASE = 1 << 30


def front_lengths(wd):
    s, c = STEP[wd], COVER[wd]
    fr = {1, 2, 3, 4, 5, 8, 17, 4 * wd - 1, 4 * wd, 4 * wd + 1, c - 1, c}
    for k in range(1, 15):
        fr |= {k * s + 4 * wd - 1, k * s + 4 * wd, k * s + 4 * wd + 1}
    return sorted(x for x in fr if 1 <= x <= c)


def routed_lengths():
    """(L, wd) for lengths whose packed batch the product routes to fcs_segw_kernel<wd>."""
    out = []
    for wd in COVER:
        for m in range(2, 9):
            for lf in front_lengths(wd):
                L = COVER[wd] * (m - 1) + lf
                if na.fixed_route(BASE, L, L, 1 << 20) == f"segment:{wd}":
                    out.append((L, wd))
    return out


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


def test_every_width_is_routed():
    na.load()
    got = {wd for _, wd in routed_lengths()}
    assert got, "no length routes to the wide-window segment kernel"


def test_segw_front_edges(dev, oracle):
    """Every routed length: packed and gapped strides, partial units, unaligned bases; the launch
    is the routed kernel."""
    cases = routed_lengths()
    assert cases
    for L, wd in cases:
        for gap, n, lead in ((0, 13, 0), (3, 6, 1), (1001, 5, 2)):
            stride = L + gap
            host = np.random.default_rng(L * 5 + gap).integers(0, 256, n * stride + 16, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            got = run(dev, d, lead, stride, L, n)
            exp = oracle_fixed(oracle, host[lead:], stride, L, n)
            assert np.array_equal(got, exp), (L, wd, stride, n, lead, int(np.argmax(got != exp)))
            assert na.last_fixed_launch() == f"segment:{wd}/768", (L, wd, na.last_fixed_launch())


def test_segw_many_units(dev, oracle):
    """Every routed width: more units than the grid's waves (the dynamic schedule), twice (the
    counter ring reused)."""
    routed = routed_lengths()
    for wd in sorted({w for _, w in routed}):
        cases = [L for L, w in routed if w == wd]
        _many_units(dev, oracle, wd, cases[len(cases) // 2])


def _many_units(dev, oracle, wd, L):
    stride = L + 7
    n = max(20001, (200 << 20) // stride)
    host = np.random.default_rng(L + wd).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[3:], stride, L, n)
    for _ in range(2):
        got = run(dev, d, 3, stride, L, n)
        assert np.array_equal(got, exp), (L, int(np.argmax(got != exp)))


def test_segw_verify_mode(dev):
    """Every routed width: RX residue check through the kernel, frames carrying their FCS, a few
    corrupted."""
    routed = routed_lengths()
    for wd in sorted({w for _, w in routed}):
        _verify(dev, [L for L, w in routed if w == wd][-1])


def _verify(dev, L):
    n = 2051
    rng = np.random.default_rng(L)
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    for i in range(n):
        f = host[i * L:i * L + L - 4].tobytes()
        host[i * L + L - 4:i * L + L] = np.frombuffer(struct.pack("<I", zlib.crc32(f)), dtype=np.uint8)
    bad_idx = sorted(set(int(x) for x in rng.integers(0, n, 19)) | {0, n - 1})
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
