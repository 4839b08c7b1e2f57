"""CPU replay of the kernel's arithmetic (tests/kernel_model.py) against the golden fixtures.

Validates the constant tables the product library builds (fcs_tables_blob), the v_perm LDS
addressing, front-lane init/masking, segment jumps and lane shifts — without a GPU."""
import random
import zlib

import numpy as np

import pytest

import kernel_model as km  # noqa: E402

na = pytest.importorskip("nstack_amd")


@pytest.fixture(scope="module")
def lds():
    return km.build_lds(na.tables_blob())


def test_blob_slice_tables_match_reference_polynomial(lds):
    blob = na.tables_blob()
    # T0 is the byte-wise table of the reflected polynomial 0xEDB88320
    for b in (0, 1, 128, 255):
        r = b
        for _ in range(8):
            r = (r >> 1) ^ (0xEDB88320 if r & 1 else 0)
        assert blob[b] == r


def test_model_on_golden_vectors(lds, golden):
    arena = golden["arena"]
    frames = golden["vectors"]["frames"]
    for fr in frames[::3]:
        assert km.model_frame(lds, arena, fr["off"], fr["len"]) == fr["crc"], fr


def test_model_edges_and_alignment(lds):
    rng = random.Random(9)
    mem = bytes(rng.randrange(256) for _ in range(12000))
    for L in (0, 1, 3, 4, 47, 48, 49, 70, 1488, 1489, 1514, 1518, 1536, 1537, 3073, 9000):
        for S in (0, 1, 2, 3, 12000 - L):
            if 0 <= S and S + L <= len(mem):
                assert km.model_frame(lds, mem, S, L) == zlib.crc32(mem[S:S + L]), (L, S)


def _shift(s, n):
    """A_n: the CRC register advanced over n zero bytes (reflected 0xEDB88320)."""
    for _ in range(n):
        for _ in range(8):
            s = (s >> 1) ^ (0xEDB88320 if s & 1 else 0)
    return s


def test_flat_kernel_chunk_shift_tables():
    """The flat variable-length kernel's C_c = A_{96c} nibble tables (fcs_tables.hpp kBlobFlat,
    136-dword stride per c): chunk_shift(s, c) = XOR_t C_c[t][nibble_t(s)] must equal A_{96c}(s)."""
    blob = na.tables_blob()
    flat = km.BLOB_INV + km.CHUNK + 8 * 16   # kBlobM768 + 8 * 16
    rng = random.Random(4)
    for c in (0, 1, 5, 15):
        for _ in range(3):
            s = rng.getrandbits(32)
            v = 0
            for t in range(8):
                v ^= int(blob[flat + c * 136 + t * 16 + ((s >> (4 * t)) & 15)])
            assert v == _shift(s, 96 * c), (c, hex(s))


def test_single_frame_kernel_decomposition():
    """fcs_one_kernel (drop-in ether_fcs, frames <= 1536 B): the frame right-aligned in a 1536-B
    window with zeros in front, 64 lanes x 24 B from a zero register, a six-level lane tree with
    A_{24*2^k}, and the all-ones start added back as A_len(0xFFFFFFFF). Replayed here with tables
    built from the polynomial alone, against zlib (= the reference ether_fcs)."""
    import zlib
    poly = 0xEDB88320
    t0 = []
    for b in range(256):
        r = b
        for _ in range(8):
            r = (r >> 1) ^ (poly if r & 1 else 0)
        t0.append(r)
    T = [t0]
    for k in range(1, 4):
        T.append([(T[k - 1][b] >> 8) ^ t0[T[k - 1][b] & 0xFF] for b in range(256)])

    def zshift(s, n):
        for _ in range(n):
            s = (s >> 8) ^ t0[s & 0xFF]
        return s

    nib = [[[zshift(e << (4 * t), 24 << k) for e in range(16)] for t in range(8)] for k in range(6)]

    def a_shift(k, x):
        v = 0
        for t in range(8):
            v ^= nib[k][t][(x >> (4 * t)) & 15]
        return v

    rng = np.random.default_rng(3)
    for L in (0, 1, 5, 60, 64, 333, 1514, 1518, 1535, 1536):
        frame = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        win = np.frombuffer(bytes(1536 - L) + frame, dtype="<u4")
        x = []
        for j in range(64):
            w = [int(v) for v in win[6 * j:6 * j + 6]]
            s = w[0]
            for i in range(6):
                s = T[3][s & 0xFF] ^ T[2][(s >> 8) & 0xFF] ^ T[1][(s >> 16) & 0xFF] ^ T[0][s >> 24] ^ (w[i + 1] if i < 5 else 0)
            x.append(s)
        for k in range(6):
            d = 1 << k
            y = [x[j] if j & d else a_shift(k, x[j]) for j in range(64)]
            x = [y[j] ^ y[j ^ d] for j in range(64)]
        got = ~(x[0] ^ zshift(0xFFFFFFFF, L)) & 0xFFFFFFFF
        assert got == zlib.crc32(frame), L


@pytest.fixture(scope="module")
def lds_dma():
    blob = na.tables_blob()
    return {ch: km.build_lds_dma(blob, ch) for ch in (2, 3, 4, 6)}


@pytest.mark.parametrize("chains", [2, 3, 4, 6])
@pytest.mark.parametrize("flen,extra", [(1496, 0), (1514, 4), (1518, 0), (1518, 2), (1520, 0), (1524, 0), (1524, 12)])
def test_dma_kernel_model(lds_dma, flen, extra, chains):
    """fcs_dma_kernel's decomposition (32 KiB slice tables looked up in per-group byte order, 6 KiB slots clamped
    at the arena end, 92-B chunks at c = 3/7/11, front mask and INV of lane 15, the chains and
    their one-step merge for every FCS_DMA_CHAINS value, A_{e_c} lane shift)
    replayed on the CPU for every item of small batches at all four base alignments, against zlib."""
    stride = flen + extra
    rng = random.Random(flen * 31 + extra + chains)
    garbage = bytes(rng.randrange(256) for _ in range(128))
    for b0 in (0, 1, 2, 3):
        n = 11
        mem = bytes(rng.randrange(256) for _ in range(b0 + n * stride + 64))
        for f in range(0, n, 4):
            got = km.model_dma_item(lds_dma[chains], mem, b0, stride, flen, n, f, garbage, chains)
            for g in range(4):
                if f + g < n:
                    S = b0 + (f + g) * stride
                    assert got[g] == zlib.crc32(mem[S:S + flen]), (flen, extra, b0, f + g)


def test_dma_windows_bank_distinct():
    """The 16 windows of a frame start on 16 distinct dword banks (mod 32), for any frame end."""
    for E in range(0, 64, 4):
        banks = {((E - km.dma_end_off(c) - 96) // 4) % 32 for c in range(16)}
        assert len(banks) == 16


def test_dma_table_lookups_bank_distinct():
    """Every table lookup of a 32-lane group hits 32 distinct banks (dword address mod 32, the
    ds_read_b32 banking), whatever words the lanes hold."""
    rng = random.Random(4)
    for _ in range(200):
        xs = [rng.getrandbits(32) for _ in range(32)]
        for k in range(4):
            assert len({km.l8_banks(l, xs[l], k) for l in range(32)}) == 32


@pytest.mark.parametrize("L", [1525, 1530, 2000, 3048, 3049, 4573, 9000, 10000])
def test_segil_decomposition_model(lds_dma, L):
    """fcs_segil_kernel's decomposition: a front segment of L - 1524 (m - 1) bytes with per-lane
    front masks and INV at the frame's first byte, then 1524-B segments whose lane 15 starts from
    the frame's CRC state after the previous segment (no shift tables between segments), reproduces
    the CRC (zlib = src/ether_fcs.c:4-19); the cover bytes before the frame are random garbage."""
    rng = np.random.default_rng(L + 2)
    frame = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
    garbage = rng.integers(0, 256, 1524, dtype=np.uint8).tobytes()
    assert km.model_segil_frame(lds_dma[2], frame, garbage) == zlib.crc32(frame)


@pytest.fixture(scope="module")
def lds_wide():
    blob = na.tables_blob()
    return {**{wd: km.build_lds_wide(blob, wd) for wd in (26, 30, 32, *km.WIDE_MID)},
            **{(wd, 8): km.build_lds_wide(blob, wd, 8) for wd in km.WIDE8},
            **{(wd, 4): km.build_lds_wide(blob, wd, 4) for wd in km.WIDE4}}


@pytest.mark.parametrize("flen,extra,wd", [(1525, 0, 32), (1530, 3, 32), (1536, 0, 32), (1537, 1, 32), (1600, 0, 32),
                                           (1611, 16, 32), (1736, 0, 32), (1737, 5, 32), (1860, 0, 32), (1861, 2, 32),
                                           (1949, 0, 32), (1950, 100, 32), (1987, 0, 32), (1988, 0, 32),
                                           (1988, 74, 32),   # 3 stride + len = 8174: the largest item a slot takes
                                           (1537, 0, 26), (1538, 3, 26), (1501, 0, 26), (1477, 0, 26), (1495, 7, 26), (1525, 0, 26),
                                           (1536, 1, 26), (1600, 0, 26), (1601, 1, 26),
                                           (1604, 0, 26), (1604, 178, 26),   # 7150: the 7 KiB slot's largest
                                           (1605, 0, 30), (1700, 1, 30), (1741, 0, 30), (1742, 2, 30), (1787, 0, 30),
                                           (1600, 3, 30)] +
                         # mid-length widths (6 KiB slots): each width's narrowest and widest frame,
                         # a gap, and the largest stride a 6 KiB slot takes (3 stride + len = 6126)
                         [(L, x, wd) for wd in km.WIDE_MID
                          for L in sorted({km.wide_cover(wd), max(870, km.wide_cover(wd) - 63)})
                          if km.wide_mid_wd(L) == wd
                          for x in (0, 5, (6126 - L) // 3 - L)])
def test_wide_kernel_model(lds_wide, flen, extra, wd):
    """fcs_wide_kernel's decomposition (128-B windows ending 124 c before the frame end, every
    live lane but the front one masking its first word, the front lane cf = (len - 1) / 124 masking
    its zc leading bytes and starting from INV[zc], lanes past it dropped, two 16-word chains merged
    with A_64, lane shift A_{124 c}, 8 KiB slots clamped at the arena end) replayed on the CPU for
    every item of small batches at all four base alignments, against zlib."""
    stride = flen + extra
    rng = random.Random(flen * 37 + extra)
    garbage = bytes(rng.randrange(256) for _ in range(2048 + 64))
    for b0 in (0, 1, 2, 3):
        n = 11
        mem = bytes(rng.randrange(256) for _ in range(b0 + n * stride + 64))
        for f in range(0, n, 4):
            got = km.model_wide_item(lds_wide[wd], mem, b0, stride, flen, n, f, garbage, wd)
            for g in range(4):
                if f + g < n:
                    S = b0 + (f + g) * stride
                    assert got[g] == zlib.crc32(mem[S:S + flen]), (flen, extra, b0, f + g)


@pytest.mark.parametrize("flen,extra", [(300, 0), (324, 1), (325, 0), (356, 0), (400, 0), (421, 3), (452, 0),
                                        (484, 0), (485, 1), (548, 0), (580, 2), (612, 2), (613, 0), (676, 0),
                                        (700, 5), (708, 0), (740, 0), (741, 0), (800, 7), (836, 0), (868, 0),
                                        (740, (6126 - 740) // 7 - 740), (868, (7150 - 868) // 7 - 868)])
def test_wide8_kernel_model(lds_wide, flen, extra):
    """fcs_wide_kernel<WD, 8>: eight frames per item, eight windows per frame (front lane
    cf = min(7, (len - 1) / (4 WD - 4))), the lane tables A_{(4 WD - 4) (slot mod 8)}, the
    eight-lane sums; replayed on the CPU for every item of small batches at four base alignments
    (the last cases: the largest stride a 6 KiB / 7 KiB slot takes), against zlib."""
    wd = km.wide8_wd(flen)
    stride = flen + extra
    rng = random.Random(flen * 41 + extra)
    garbage = bytes(rng.randrange(256) for _ in range(2048 + 64))
    for b0 in (0, 1, 2, 3):
        n = max(19, 2 * km.wide_slot(wd) // stride + 3)   # the host takes arenas of two slots or more
        mem = bytes(rng.randrange(256) for _ in range(b0 + n * stride + 64))
        for f in range(0, n, 8):
            got = km.model_wide_item(lds_wide[(wd, 8)], mem, b0, stride, flen, n, f, garbage, wd, 8)
            for g in range(8):
                if f + g < n:
                    S = b0 + (f + g) * stride
                    assert got[g] == zlib.crc32(mem[S:S + flen]), (flen, extra, b0, f + g)


@pytest.mark.parametrize("flen,extra", [(130, 0), (132, 1), (133, 0), (148, 0), (180, 3), (200, 0), (244, 0),
                                        (245, 2), (256, 0), (300, 5), (324, 0), (340, 0), (356, 1), (388, 0),
                                        (399, 0), (404, 0), (372, (6126 - 372) // 15 - 372),
                                        (399, (7150 - 399) // 15 - 399)])
def test_wide4_kernel_model(lds_wide, flen, extra):
    """fcs_wide_kernel<WD, 4>: sixteen frames per item, four windows per frame (front lane
    cf = min(3, (len - 1) / (4 WD - 4))), lane tables A_{(4 WD - 4) (slot mod 4)}, the quad sums;
    replayed on the CPU for every item at four base alignments, against zlib."""
    wd = km.wide4_wd(flen)
    stride = flen + extra
    rng = random.Random(flen * 43 + extra)
    garbage = bytes(rng.randrange(256) for _ in range(2048 + 64))
    for b0 in (0, 1, 2, 3):
        n = max(35, 2 * km.wide_slot(wd) // stride + 3)   # the host takes arenas of two slots or more
        mem = bytes(rng.randrange(256) for _ in range(b0 + n * stride + 64))
        for f in range(0, n, 16):
            got = km.model_wide_item(lds_wide[(wd, 4)], mem, b0, stride, flen, n, f, garbage, wd, 4)
            for g in range(16):
                if f + g < n:
                    S = b0 + (f + g) * stride
                    assert got[g] == zlib.crc32(mem[S:S + flen]), (flen, extra, b0, f + g)


def test_wide8_windows_bank_distinct():
    """The eight windows of a frame in fcs_wide_kernel<WD, 8> start on eight distinct dword banks."""
    for wd in km.WIDE8:
        for E in range(0, 64, 4):
            assert len({((E - km.wide_end_off(c, wd) - 4 * wd) // 4) % 32 for c in range(8)}) == 8


def test_wide_windows_bank_distinct():
    """The 16 windows of a frame in fcs_wide_kernel start on 16 distinct dword banks (mod 32)."""
    for wd in (26, 30, 32, *km.WIDE_MID):
        for E in range(0, 64, 4):
            banks = {((E - km.wide_end_off(c, wd) - 4 * wd) // 4) % 32 for c in range(16)}
            assert len(banks) == 16


@pytest.mark.parametrize("L,wd", [(1989, 26), (3100, 26), (3208, 26), (3209, 26), (6100, 26), (9216, 26),
                                  (1989, 30), (3720, 30), (3721, 30), (5000, 30), (9216, 30), (9300, 30), (9301, 30),
                                  (2000, 18), (2184, 18), (2185, 18), (2200, 19), (2500, 22), (2696, 22), (4000, 22),
                                  (2800, 23), (2824, 23), (3049, 26), (65536, 32)])
def test_segw_decomposition_model(lds_wide, L, wd):
    """fcs_segw_kernel<WD>'s decomposition: a front segment of L - C (m - 1) bytes (C = the wide
    kernel's cover 15 (4 WD - 4) + 4 WD: 1092 B for WD 18 ... 1988 B for WD 32) with the wide kernel's front lane, then
    C-byte segments whose lane 15 starts unmasked from the frame's CRC state after the previous
    segment, reproduces the CRC (zlib = src/ether_fcs.c:4-19); cover bytes before the frame are
    random garbage."""
    rng = np.random.default_rng(L * 3 + wd)
    frame = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
    garbage = rng.integers(0, 256, 2048, dtype=np.uint8).tobytes()
    assert km.model_segw_frame(lds_wide[wd], frame, garbage, wd) == zlib.crc32(frame)


@pytest.mark.parametrize("seed,lead", [(1, 0), (2, 5), (3, 15), (4, 1)])
def test_inet_stream_attribution(seed, lead):
    """inet_stream_kernel's attribution of a packed window's bytes to its packets (lane regions of
    96 B, one packet start per 16-B piece, dot4 running sums split at a start) gives every packet
    exactly its own even/odd byte sums E + 256 O, the word sum the checksum folds (the RFC 1071
    sum of src/ip.c:39-62 before the fold). Packets of 16 B to 9 KiB, a window spanning several
    6 KiB items, a partial window, and every start alignment within the first piece."""
    rng = np.random.default_rng(seed)
    npk = 64 if seed != 4 else 37
    ln = rng.choice([16, 17, 20, 31, 64, 65, 576, 1518], npk)
    ln[rng.integers(0, npk, 3)] = rng.integers(2000, 9000, 3)
    starts = lead + np.concatenate([[0], np.cumsum(ln)[:-1]])
    total = int(starts[-1] + ln[-1])
    span = rng.integers(0, 256, total + 16, dtype=np.uint8).tobytes()
    got = km.model_inet_window(span, [int(s) for s in starts], total)
    for i in range(npk):
        pk = span[int(starts[i]):int(starts[i]) + int(ln[i])]
        e = sum(pk[j] for j in range(len(pk)) if (int(starts[i]) + j) % 2 == 0)
        o = sum(pk[j] for j in range(len(pk)) if (int(starts[i]) + j) % 2 == 1)
        assert got[i] == e + 256 * o, i
    assert all(v == 0 for v in got[npk:])
