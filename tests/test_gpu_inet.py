"""GPU parity of the Internet-checksum kernels (include/nstack_inet.h) through the
C ABI, against the oracle (oracle/inet_oracle.c: ip.c:39-62, tcp.c:167-213, udp.c:136-174) and
the golden fixtures. Bit-exact is the bar. The oracle's own pinning (RFC known answers plus an
independent RFC 1071 witness; no reference build) is described in tests/test_inet_oracle.py."""
import struct
import threading

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MODES = ("ip", "tcp", "udp")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    na.load()
    return torch.device("cuda:0")


@pytest.fixture(params=["group", "flat", "dma"])
def inet_kernel(request):
    """Run a test through every kernel (identical results required): group = one 16-lane group
    per packet (small batches), flat = packets dealt to lanes by size, dma = fixed-stride packets
    four to a wave item through LDS (where their geometry fits its slots, else flat)."""
    old = na.inet_set_flat_threshold((1 << 63) if request.param == "group" else 0)
    old_dma = na.inet_set_dma_threshold(0 if request.param == "dma" else (1 << 63))
    yield request.param
    na.inet_set_flat_threshold(old)
    na.inet_set_dma_threshold(old_dma)


def to_dev(arr: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(arr)).to(dev)


def oracle_batch(o, mode, arena: np.ndarray, off, ln, addr):
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(ln, dtype=np.uint32)
    out = np.empty(len(off), dtype=np.uint16)
    a = None if addr is None else np.ascontiguousarray(addr, dtype=np.uint32)
    o.oracle_inet_batch(na.INET_MODES[mode], arena.ctypes.data, off.ctypes.data, ln.ctypes.data,
                        None if a is None else a.ctypes.data, out.ctypes.data, len(off))
    return out


def run_batch_dev(dev, mode, arena: np.ndarray, off, ln, addr):
    d_arena = to_dev(arena, dev)
    d_off = to_dev(np.asarray(off, dtype=np.uint64).view(np.int64), dev)
    d_len = to_dev(np.asarray(ln, dtype=np.uint32).view(np.int32), dev)
    d_addr = None if addr is None else to_dev(np.asarray(addr, dtype=np.uint32).view(np.int32), dev)
    out = torch.empty(len(off), dtype=torch.int16, device=dev)
    na.inet_batch_dev(mode, d_arena, arena.nbytes, d_off, d_len, d_addr, out, len(off))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint16)


def golden_groups(g):
    arena = np.frombuffer(g["arena_bytes"], dtype=np.uint8).copy()
    for mode in MODES:
        recs = [r for r in g["packets"] if r["mode"] == mode]
        off = np.array([r["off"] for r in recs], dtype=np.uint64)
        ln = np.array([r["len"] for r in recs], dtype=np.uint32)
        addr = np.array([[r["src"], r["dst"]] for r in recs], dtype=np.uint32).reshape(-1)
        exp = np.array([r["expect"] for r in recs], dtype=np.uint16)
        yield mode, arena, off, ln, (None if mode == "ip" else addr), exp, recs


def test_golden_batch_dev(dev, inet_golden, inet_kernel):
    for mode, arena, off, ln, addr, exp, recs in golden_groups(inet_golden):
        got = run_batch_dev(dev, mode, arena, off, ln, addr)
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, [(recs[i]["tag"], recs[i]["len"], recs[i]["off"] % 16, hex(got[i]), hex(exp[i]))
                               for i in bad[:10]]


def test_golden_batch_host(dev, inet_golden, inet_kernel):
    for mode, arena, off, ln, addr, exp, _ in golden_groups(inet_golden):
        out = np.zeros(len(off), dtype=np.uint16)
        na.inet_batch_host(mode, arena, arena.nbytes, off, ln, addr, out, len(off))
        assert np.array_equal(out, exp), mode


def test_known_answers_single(dev, inet_golden):
    for k in inet_golden["kat"]:
        b = bytes.fromhex(k["hex"])
        assert struct.pack("<H", na.ip_checksum(b)).hex() == k["expect_wire"], k


def test_single_forms_match_oracle(dev, inet_oracle):
    rng = np.random.default_rng(5)
    for n in (0, 1, 2, 3, 20, 21, 60, 1480, 1481, 9000):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s, d = (int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64))
        assert na.ip_checksum(b) == inet_oracle.oracle_ip_checksum(b, n)
        assert na.tcp_checksum(s, d, b) == inet_oracle.oracle_tcp_checksum(s, d, b, n)
        assert na.udp_checksum(b, s, d) == inet_oracle.oracle_udp_checksum(b, n, s, d)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("start,stride,L", [(14, 1518, 1500), (34, 1518, 1480), (14, 1518, 20),
                                             (0, 1500, 1500), (1, 97, 61), (3, 9000, 8997), (5, 64, 0),
                                             (7, 1532, 1532), (2, 120, 64), (6, 1024, 1000), (9, 2048, 1024), (1, 1519, 1517),
                                             (3, 64, 64), (15, 33, 33), (1, 20, 1), (2, 4096, 40)])
def test_fixed_dev_vs_oracle(dev, inet_oracle, mode, start, stride, L, inet_kernel):
    """Fixed-stride packets inside frames: the IP datagram at +14, the TCP segment at +34, the IP
    header alone, odd strides/starts (every alignment), jumbo, empty packets, and packets of up to
    64 B at tight and wide strides (the lane-per-packet kernel in the large-batch kernels' runs)."""
    n = 6000
    rng = np.random.default_rng(start * 7 + L)
    host = rng.integers(0, 256, start + n * stride + 16, dtype=np.uint8)
    addr = rng.integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    d = to_dev(host, dev)
    d_addr = to_dev(addr.view(np.int32), dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    na.inet_fixed_dev(mode, d.data_ptr() + start, stride, L, n, None if mode == "ip" else d_addr, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    off = start + np.arange(n, dtype=np.uint64) * stride
    exp = oracle_batch(inet_oracle, mode, host, off, np.full(n, L, np.uint32), None if mode == "ip" else addr)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("mode", MODES)
def test_random_var_vs_oracle(dev, inet_oracle, mode, inet_kernel):
    """20k packets, random lengths 0..3000 (IMIX-heavy), random (overlapping) offsets."""
    rng = np.random.default_rng(11 + len(mode))
    n = 20000
    arena = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    ln = rng.choice([0, 1, 20, 40, 64, 576, 1480, 1500], n).astype(np.uint32)
    ln[::7] = rng.integers(0, 3000, len(ln[::7]))
    off = rng.integers(0, arena.size - 3001, n).astype(np.uint64)
    addr = rng.integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    a = None if mode == "ip" else addr
    got = run_batch_dev(dev, mode, arena, off, ln, a)
    assert np.array_equal(got, oracle_batch(inet_oracle, mode, arena, off, ln, a))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("lead", [0, 1, 3])
def test_packed_var_windows(dev, inet_oracle, mode, lead, inet_kernel):
    """Packed variable batches (each packet starts where the previous ends), as the LDS stream takes
    them window by window (64 packets): IMIX lengths, 16-B packets, long ones spanning several 6 KiB
    items, and windows the stream hands to its flat path (a gap, an overlap, a packet under 16 B, an
    empty one), at every base alignment."""
    rng = np.random.default_rng(100 + lead + 7 * len(mode))
    n = 64 * 60 + 17
    ln = rng.choice([16, 17, 63, 64, 65, 576, 1500, 1518], n).astype(np.int64)
    ln[64 * 5:64 * 6] = rng.integers(3000, 9000, 64)      # a window of long packets (many items)
    ln[64 * 7 + 9] = 15                                     # a short packet: flat window
    ln[64 * 9 + 40] = 0                                     # an empty packet: flat window
    off = lead + np.concatenate([[0], np.cumsum(ln)[:-1]])
    off[64 * 11 + 3:] += 5                                  # a gap: flat window
    off[64 * 13 + 50] -= 8                                  # an overlap: flat window
    arena = rng.integers(0, 256, int(off[-1] + ln[-1]) + 64, dtype=np.uint8)
    arena[int(off[64 * 15]):int(off[64 * 15]) + 2000] = 0  # all-zero packets
    addr = rng.integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    a = None if mode == "ip" else addr
    got = run_batch_dev(dev, mode, arena, off.astype(np.uint64), ln.astype(np.uint32), a)
    assert np.array_equal(got, oracle_batch(inet_oracle, mode, arena, off, ln, a))


@pytest.mark.parametrize("mode", MODES)
def test_short_var_packets(dev, inet_oracle, mode, inet_kernel):
    """Variable batches of packets of 0..64 B at scattered and overlapping offsets (IP headers of a
    TX batch; the stream kernel's lane-per-packet windows), one window with a longer packet (its
    flat path), every alignment."""
    rng = np.random.default_rng(300 + len(mode))
    n = 64 * 40 + 5
    ln = rng.integers(0, 65, n).astype(np.uint32)
    ln[::97] = 64
    ln[64 * 7 + 3] = 65                                     # one window on the flat path
    arena = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    off = rng.integers(0, arena.size - 80, n).astype(np.uint64)
    addr = rng.integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    a = None if mode == "ip" else addr
    got = run_batch_dev(dev, mode, arena, off, ln, a)
    assert np.array_equal(got, oracle_batch(inet_oracle, mode, arena, off, ln, a))


def test_quirks(dev, inet_oracle, inet_kernel):
    """nstack-specific results: all-zero data (acc = 0xffff start), sums that are a nonzero
    multiple of 0xffff, the htons(len) truncation above 64 KiB, and headers that verify to 0."""
    cases = [bytes(40), b"\xff\xff", b"\xff\xff" * 3, b"\x00\x01\xff\xfe", bytes(1), b"\xff"]
    for b in cases:
        assert na.ip_checksum(b) == inet_oracle.oracle_ip_checksum(b, len(b)), b.hex()
    assert na.ip_checksum(bytes(40)) == 0
    big = np.random.default_rng(1).integers(0, 256, 70000, dtype=np.uint8).tobytes()
    assert na.tcp_checksum(1, 2, big) == inet_oracle.oracle_tcp_checksum(1, 2, big, len(big))
    assert na.udp_checksum(big, 3, 4) == inet_oracle.oracle_udp_checksum(big, len(big), 3, 4)
    hdr = bytearray(np.random.default_rng(2).integers(0, 256, 20, dtype=np.uint8).tobytes())
    hdr[10:12] = b"\0\0"
    hdr[10:12] = struct.pack("<H", na.ip_checksum(bytes(hdr)))   # ip_hton, src/ip.c:79-80
    assert na.ip_checksum(bytes(hdr)) == 0                        # the check of src/ip.c:151


def test_concurrent_single_callers(dev, inet_oracle):
    errs = []

    def worker(seed):
        rng = np.random.default_rng(seed)
        for _ in range(30):
            b = rng.integers(0, 256, int(rng.integers(0, 2000)), dtype=np.uint8).tobytes()
            if na.ip_checksum(b) != inet_oracle.oracle_ip_checksum(b, len(b)):
                errs.append(seed)

    th = [threading.Thread(target=worker, args=(s,)) for s in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs


def test_large_fixed_sampled(dev, inet_oracle, oracle, inet_kernel):
    """4 M TCP segments (+34, 1480 B) inside device-generated 1518-B frames: 3000 sampled
    packets against the oracle, and two half launches equal one launch."""
    n, stride, start, L = 4 << 20, 1518, 34, 1480
    nbytes = n * stride + 64
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(buf, nbytes, 0x1E7, 0)
    addr = torch.randint(-2**31, 2**31 - 1, (2 * n,), dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    na.inet_fixed_dev("tcp", buf.data_ptr() + start, stride, L, n, addr, out)
    half = torch.empty(n, dtype=torch.int16, device=dev)
    h = n // 2
    na.inet_fixed_dev("tcp", buf.data_ptr() + start, stride, L, h, addr, half)
    na.inet_fixed_dev("tcp", buf.data_ptr() + start + h * stride, stride, L, n - h, addr[2 * h:], half[h:])
    torch.cuda.synchronize()
    assert torch.equal(out, half)
    got = out.cpu().numpy().view(np.uint16)
    a = addr.cpu().numpy().view(np.uint32)
    idx = np.unique(np.concatenate([np.random.default_rng(9).integers(0, n, 3000), [0, n - 1]]))
    p = np.empty(L, dtype=np.uint8)
    for i in idx:   # regenerate the packet's bytes on the host (counter-based generator)
        oracle.oracle_splitmix_fill(p.ctypes.data, L, 0x1E7, int(start + i * stride))
        assert got[i] == inet_oracle.oracle_tcp_checksum(int(a[2 * i]), int(a[2 * i + 1]), p.ctypes.data, L), i


@pytest.mark.parametrize("n", [1, 3, 4, 5, 63, 64, 65, 257, 4099, 70001])
def test_dma_partial_items(dev, inet_oracle, n):
    """The fixed-stride LDS-DMA kernel at batch sizes that leave a partial last item (n mod 4) and
    uneven dynamic chunks, on 1518-B strides at an odd start (the IP datagram of frames packed at an
    odd address), against the oracle for every packet."""
    old = na.inet_set_dma_threshold(0)
    try:
        _dma_partial_items(dev, inet_oracle, n)
    finally:
        na.inet_set_dma_threshold(old)


def _dma_partial_items(dev, inet_oracle, n):
    start, stride, L = 15, 1518, 1500
    rng = np.random.default_rng(n)
    host = rng.integers(0, 256, start + (n - 1) * stride + L, dtype=np.uint8)
    addr = rng.integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    d = to_dev(host, dev)
    d_addr = to_dev(addr.view(np.int32), dev)
    off = start + np.arange(n, dtype=np.uint64) * stride
    for mode in MODES:
        out = torch.empty(n, dtype=torch.int16, device=dev)
        na.inet_fixed_dev(mode, d.data_ptr() + start, stride, L, n, None if mode == "ip" else d_addr, out)
        torch.cuda.synchronize()
        exp = oracle_batch(inet_oracle, mode, host, off, np.full(n, L, np.uint32), None if mode == "ip" else addr)
        assert np.array_equal(out.cpu().numpy().view(np.uint16), exp), mode


def test_argument_errors(dev):
    with pytest.raises(na.FcsError):
        na.inet_fixed_dev(9, 64, 20, 20, 1, None, 64)
    with pytest.raises(na.FcsError):
        na.inet_fixed_dev("udp", 64, 20, 20, 1, None, 64)
    with pytest.raises(na.FcsError):
        na.inet_fixed_dev("ip", 64, 10, 20, 2, None, 64)   # stride < len


def _dev_digest(out):
    """Sum of the u16 results and sum of result * (i & 0xffff), on the device (as the oracle's)."""
    u = out.to(torch.int64) & 0xFFFF
    idx = torch.arange(out.numel(), device=out.device, dtype=torch.int64) & 0xFFFF
    return int(u.sum().item()), int((u * idx).sum().item())


def _oracle_digest(inet_oracle, mode, seed, off, ln, addr, n):
    import ctypes
    s, w = ctypes.c_uint64(), ctypes.c_uint64()
    inet_oracle.oracle_inet_splitmix_digest(mode, seed, off.ctypes.data, ln.ctypes.data, 0, 0,
                                            None if addr is None else addr.ctypes.data, n, 16,
                                            ctypes.byref(s), ctypes.byref(w))
    return s.value, w.value


def test_full_imix_digest(dev, inet_oracle):
    """Every checksum of 128 M packed IMIX packets (7:4:1 of 64/576/1518 B, shuffled; the LDS
    stream kernel), against the oracle's digest of the same splitmix stream (16 host threads,
    packets regenerated on the fly)."""
    n = 128 << 20
    c1518, c576 = n // 12, (n * 4) // 12
    ln = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), [n - c576 - c1518, c576, c1518])
    np.random.default_rng(7).shuffle(ln)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1], dtype=np.uint64, out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    arena = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, total + 64, 0x17A5, 0)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    na.inet_batch_dev("ip", arena, total + 64, d_off, d_len, None, out, n)
    torch.cuda.synchronize()
    got = _dev_digest(out)
    del arena, d_off, d_len, out
    torch.cuda.empty_cache()
    assert got == _oracle_digest(inet_oracle, 0, 0x17A5, off, ln, None, n)


@pytest.mark.parametrize("mode,start,L", [("tcp", 34, 1480), ("ip", 14, 20)])
def test_full_fixed_digest(dev, inet_oracle, mode, start, L):
    """Every checksum of 64 M packets of packed 1518-B frames: TCP segments (+34, 1480 B; the
    LDS-DMA fixed-stride kernel) and IP headers (+14, 20 B; the lane-per-packet kernel), against
    the oracle's digest of the same stream and addresses."""
    n, stride = 64 << 20, 1518
    nbytes = n * stride + 64
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(buf, nbytes, 0x7C9, 0)
    addr = np.random.default_rng(5).integers(0, 2**32, 2 * n, dtype=np.uint64).astype(np.uint32)
    d_addr = torch.from_numpy(addr.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    na.inet_fixed_dev(mode, buf.data_ptr() + start, stride, L, n, d_addr if mode != "ip" else None, out)
    torch.cuda.synchronize()
    got = _dev_digest(out)
    del buf, d_addr, out
    torch.cuda.empty_cache()
    off = start + np.arange(n, dtype=np.uint64) * np.uint64(stride)
    ln = np.full(n, L, dtype=np.uint32)
    m = {"ip": 0, "tcp": 1, "udp": 2}[mode]
    assert got == _oracle_digest(inet_oracle, m, 0x7C9, off, ln, addr if m else None, n)
