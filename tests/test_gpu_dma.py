"""GPU parity of the LDS-DMA fixed kernel (fcs_dma_kernel).

Fixed-length batches of 1496..1524-B frames whose four consecutive frames fit a 6 KiB slot
(3 stride + len <= 6126) and whose arena holds two slots take this kernel, large batches of
1496..1503 B too (round 4: they took the flat kernel before); smaller ones the register-load
single kernel. Every case is checked bit-exact against the oracle (the CPU
restatement of src/ether_fcs.c:4-19), at all four base alignments, with batch sizes on both sides
of the selection threshold and grids from one partial item to many sweeps, so the slot clamping at
the arena end and frames past n in a wave's last item are exercised. Verify mode (frames carrying
their FCS trailer, RX residue check) goes through the same kernel's epilogue.
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


LENS = [1496, 1497, 1503, 1504, 1513, 1514, 1517, 1518, 1519, 1520, 1523, 1524]


@pytest.mark.parametrize("L", LENS)
def test_dma_lengths_strides_alignments(dev, oracle, L):
    strides = sorted({s for s in (L, L + 1, L + 2, L + 3, L + 10, 1536, 1544) if 3 * s + L <= 6126})
    for stride in strides:
        for n in (8, 9, 13, 257, 4099):
            host = np.random.default_rng(L * 131 + stride * 7 + n).integers(0, 256, n * stride + 8, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            for lead in (0, 1, 2, 3):
                # the last frame ends exactly at the end of the buffer the engine is told about
                out = torch.empty(n, dtype=torch.int32, device=dev)
                na.fixed_dev(d.data_ptr() + lead, stride, L, n, out)
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                exp = oracle_fixed(oracle, host[lead:], stride, L, n)
                assert np.array_equal(got, exp), (L, stride, n, lead, int(np.argmax(got != exp)))


def test_dma_many_sweeps(dev, oracle):
    """More items than the persistent grid holds (every wave walks several items)."""
    L, n = 1518, 70001
    host = np.random.default_rng(5).integers(0, 256, n * L + 3, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    for lead in (0, 3):
        out = torch.empty(n, dtype=torch.int32, device=dev)
        na.fixed_dev(d.data_ptr() + lead, L, L, n, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, oracle_fixed(oracle, host[lead:], L, L, n)), lead


@pytest.mark.parametrize("L", [1500, 1518, 1524])
def test_dma_verify_mode(dev, L):
    """RX residue check through the DMA kernel: frames of L bytes (L - 4 covered + LE FCS trailer),
    a few corrupted; ok[] and the bad count against zlib."""
    n = 20011
    rng = np.random.default_rng(L)
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    for i in range(n):
        f = host[i * L:i * L + L - 4].tobytes()
        host[i * L + L - 4:i * L + L] = np.frombuffer(struct.pack("<I", zlib.crc32(f)), dtype=np.uint8)
    bad_idx = sorted(set(int(x) for x in rng.integers(0, n, 37)) | {0, n - 1})
    for i in bad_idx:
        host[i * L + int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    d = torch.from_numpy(host).to(dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    bad = torch.zeros(1, dtype=torch.int64, device=dev)
    na.verify_fixed_dev(d, L, L, n, ok, bad)
    torch.cuda.synchronize()
    okh = ok.cpu().numpy()
    exp = np.ones(n, dtype=np.uint8)
    exp[bad_idx] = 0
    assert np.array_equal(okh, exp)
    assert int(bad.item()) == len(bad_idx)


@pytest.mark.parametrize("L,stride,lead", [(1518, 1518, 0), (1518, 1518, 3), (1514, 1518, 1), (1524, 1524, 2),
                                           (1496, 1496, 1), (1503, 1503, 3), (1500, 1536, 0)])
def test_dma_dynamic_tail(dev, oracle, L, stride, lead):
    """Batches of >= 16 items (64 frames) per wave of the grid hand the last quarter of their items out
    through the device work counter (guided chunks): every frame of a 1 M-frame batch against the
    oracle, and a second launch on the same stream reusing the counter ring."""
    n = (1 << 20) + 7
    host = np.random.default_rng(L + stride + lead).integers(0, 256, n * stride + 8, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host[lead:], stride, L, n)
    for _ in range(2):
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        na.fixed_dev(d.data_ptr() + lead, stride, L, n, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert np.array_equal(got, exp), int(np.argmax(got != exp))


def test_dma_dynamic_tail_concurrent_streams(dev, oracle):
    """Two large launches in flight on two streams take different counter slots."""
    L, n = 1518, (1 << 19) + 3
    host = np.random.default_rng(11).integers(0, 256, n * L, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host, L, L, n)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1 = torch.zeros(n, dtype=torch.int32, device=dev)
    o2 = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    na.fixed_dev(d, L, L, n, o1, s1)
    na.fixed_dev(d, L, L, n, o2, s2)
    torch.cuda.synchronize()
    assert np.array_equal(o1.cpu().numpy().view(np.uint32), exp)
    assert np.array_equal(o2.cpu().numpy().view(np.uint32), exp)


def test_counter_ring_reuse_across_streams(dev, oracle):
    """more dynamic launches in flight than the 256-slot counter ring, spread over two
    streams. A slot's new user must wait for its previous kernel before zeroing it; otherwise two
    kernels share one counter and skip each other's items (entries never written). 600 launches of
    262144 x 1518 B (the smallest batch that takes the dynamic schedule on 256 CUs), each into its
    own output, all checked against the oracle's CRCs."""
    L, n, launches = 1518, 1 << 18, 600
    host = np.random.default_rng(12).integers(0, 256, n * L, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    exp = oracle_fixed(oracle, host, L, L, n)
    outs = torch.full((launches, n), -1, dtype=torch.int32, device=dev)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    for k in range(launches):
        na.fixed_dev(d, L, L, n, outs[k], streams[k & 1])
    torch.cuda.synchronize()
    got = outs.cpu().numpy().view(np.uint32)
    bad = np.nonzero((got != exp[None, :]).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} launches with wrong or unwritten entries, first {int(bad[0])}"
