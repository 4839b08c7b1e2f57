"""Bit-level CPU model of the gfx950 FCS kernel's arithmetic (TEST INFRASTRUCTURE ONLY).

It replays, per half-wave, exactly what nstack_amd/csrc/fcs_kernel.hip does — the LDS image the
workgroup builds from the table blob, v_perm_b32 address formation, the slice-by-4 chain, the
front-lane INV injection and masking, the segment jump, the per-lane shift and the XOR reduce —
so table or layout mistakes show up on the CPU before any GPU time is spent. It is checked
against the oracle (tests/test_kernel_model.py); it is never used to produce product results.
"""
import numpy as np

CHUNK, GROUP = 96, 16
SEG = CHUNK * GROUP
LDS_LANE, LDS_JUMP, LDS_H48, LDS_H24, LDS_INV, LDS_BYTES = 131072, 147456, 147968, 148480, 148992, 149376
BLOB_SLICE, BLOB_LANE = 0, 1024
BLOB_JUMP = BLOB_LANE + 8 * 16 * 32
BLOB_H48 = BLOB_JUMP + 8 * 16
BLOB_H24 = BLOB_H48 + 8 * 16
BLOB_INV = BLOB_H24 + 8 * 16
BLOB_WORDS = BLOB_INV + CHUNK


def v_perm(s0, s1, sel):
    data = ((s0 & 0xFFFFFFFF) << 32) | (s1 & 0xFFFFFFFF)
    out = 0
    for i in range(4):
        b = (sel >> (8 * i)) & 0xFF
        if b >= 13:
            v = 0xFF
        elif b == 12:
            v = 0
        elif b < 8:
            v = (data >> (8 * b)) & 0xFF
        else:
            raise ValueError("sign-extension selectors unused")
        out |= v << (8 * i)
    return out


def build_lds(blob):
    lds = np.zeros(LDS_BYTES // 4, dtype=np.uint32)
    for i in range(8192):
        h, b, odd = i >> 12, (i >> 4) & 255, (i >> 3) & 1
        k = (2 if odd else 3) if h == 0 else (0 if odd else 1)
        lds[i * 4:i * 4 + 4] = blob[BLOB_SLICE + 256 * k + b]
    n = BLOB_WORDS - BLOB_LANE
    lds[LDS_LANE // 4:LDS_LANE // 4 + n] = blob[BLOB_LANE:BLOB_LANE + n]
    return lds


def rd(lds, addr):
    assert addr % 4 == 0 and 0 <= addr < LDS_BYTES
    return int(lds[addr // 4])


def step4(lds, x, j):
    base0, base1 = j * 4, 0x10000 | (j * 4)
    a0 = v_perm(x, base0, 0x0C020400)
    a1 = v_perm(x, base0, 0x0C020500)
    a2 = v_perm(x, base1, 0x0C020600)
    a3 = v_perm(x, base1, 0x0C020700)
    return rd(lds, a0) ^ rd(lds, a1 + 128) ^ rd(lds, a2) ^ rd(lds, a3 + 128)


def lane_shift(lds, s, j):
    lanebase = LDS_LANE | (j * 4)
    r = 0
    for t in range(8):
        sh = (s >> (4 * t - 7)) if 4 * t >= 7 else ((s << (7 - 4 * t)) & 0xFFFFFFFF)
        r ^= rd(lds, ((sh & 0x780) | lanebase) + t * 2048)
    return r


def uniform_shift(lds, s, region):
    r = 0
    for t in range(8):
        sh = (s >> (4 * t - 2)) if 4 * t >= 2 else ((s << 2) & 0xFFFFFFFF)
        r ^= rd(lds, ((sh & 0x3C) | region) + t * 64)
    return r


def jump(lds, s):
    return uniform_shift(lds, s, LDS_JUMP)


def alignbyte(hi, lo, r):
    return ((((hi << 32) | lo) >> (8 * (r & 3))) & 0xFFFFFFFF)


def model_frame(lds, mem: bytes, S: int, L: int):
    """FCS of mem[S:S+L] computed the kernel's way. mem is the whole readable arena."""
    E = S + L
    m = (L + SEG - 1) // SEG if L else 1
    state = [0] * GROUP
    lo4, hi4 = 0, (len(mem) + 3) & ~3
    padded = mem + b"\0" * 8
    for k in range(m):
        for j in range(GROUP):
            cend = E - SEG * (m - 1 - k) - CHUNK * j
            cstart = cend - CHUNK
            z = (S - cstart) if k == 0 else -1
            zr = max(-1, min(CHUNK, z))
            r = cstart & 3
            W = CHUNK // 4
            d = [0] * (W + 1)
            if zr < CHUNK:
                a = cstart & ~3
                for q in range(W + 1 if r else W):
                    ad = a + 4 * q
                    if ad >= lo4 and ad + 4 <= hi4:
                        d[q] = int.from_bytes(padded[ad:ad + 4], "little")
            w = [alignbyte(d[i + 1], d[i], r) for i in range(W)]
            if k == 0:
                for i in range(W):
                    t = max(0, min(4, zr - 4 * i))
                    w[i] &= (0xFFFFFFFFFFFFFFFF << (8 * t)) & 0xFFFFFFFF
                iv = rd(lds, LDS_INV + 4 * max(0, min(CHUNK - 1, zr)))
                x0 = iv if 0 <= zr < CHUNK else 0
            else:
                x0 = 0
            q = W // 4
            sa, sb, sc, sd = x0, 0, 0, 0
            for i in range(q):
                sa = step4(lds, sa ^ w[i], j)
                sb = step4(lds, sb ^ w[q + i], j)
                sc = step4(lds, sc ^ w[2 * q + i], j)
                sd = step4(lds, sd ^ w[3 * q + i], j)
            ab = uniform_shift(lds, sa, LDS_H24) ^ sb
            cd = uniform_shift(lds, sc, LDS_H24) ^ sd
            r = uniform_shift(lds, ab, LDS_H48) ^ cd
            state[j] = r if k == 0 else (jump(lds, state[j]) ^ r)
    v = 0
    for j in range(GROUP):
        v ^= lane_shift(lds, state[j], j)
    return (~v & 0xFFFFFFFF) if L else 0


# ---- LDS-DMA fixed kernel (fcs_dma_kernel): 32 KiB slice tables, 6 KiB slots, windows at e_c ----
BLOB_M768 = BLOB_INV + CHUNK
BLOB_FLAT = BLOB_M768 + 8 * 16
BLOB_LANE_DMA = BLOB_FLAT + 16 * 544 // 4
DMA_SLOT = 6144
DMA_COVER = 1524


def dma_end_off(c):
    return 96 * c - 4 * (c >> 2)


def dma_short_lane(c):
    return (c & 3) == 3 and c < 15


BLOB_MERGE = BLOB_LANE_DMA + 8 * 16 * 32
DMA_CHAINS = 2                    # fcs_kernel.hip FCS_DMA_CHAINS default
MERGE_HOLE, INV_HOLE = 128, 128 + 4 * 5


def hole(q):
    """Byte offset of hole q: the upper 128 B of row q of the DMA kernel's table image."""
    return q * 256 + 128


def build_lds_dma(blob, chains=DMA_CHAINS):
    """fcs_dma_kernel's 64 KiB table image (byte offsets as the kernel stages them): row e = 256 B;
    bytes [0,128) slot s = T_{3-s}[e] x 8 replicas; hole 16t+n = lane-table t nibble n for the 32
    lane slots; holes MERGE_HOLE.. the chain-merge tables A_{4 CL m}; INV after them."""
    cl = 24 // chains
    lds = np.zeros(65536 // 4, dtype=np.uint32)
    for e in range(256):
        for sl in range(4):
            lds[(e * 256 + sl * 32) // 4:(e * 256 + sl * 32) // 4 + 8] = blob[BLOB_SLICE + 256 * (3 - sl) + e]
    for i in range(4096):
        lds[(hole(i >> 5) + (i & 31) * 4) // 4] = blob[BLOB_LANE_DMA + i]
    for m in range(chains - 1):
        k = (cl // 2) * (m + 1)          # A_{8k}
        for t in range(8):
            for e in range(16):
                lds[(hole(MERGE_HOLE + 4 * m + (t >> 1)) + 64 * (t & 1) + 4 * e) // 4] = \
                    blob[BLOB_MERGE + (k - 1) * 128 + t * 16 + e]
    for z in range(96):
        lds[(hole(INV_HOLE + z // 32) + (z % 32) * 4) // 4] = blob[BLOB_INV + z]
    return lds


def step4_l8(lds, x, lane):
    """fcs_dma_kernel's step4_l8: lane group h = (lane >> 3) & 3 looks byte k ^ h up in slot k ^ h."""
    h = (lane >> 3) & 3
    r = 0
    for k in range(4):
        B = (lane & 7) * 4 + 32 * (k ^ h)
        r ^= int(lds[v_perm(x, B, 0x0C0C0400 + ((k ^ h) << 8)) // 4])
    return r


def l8_banks(lane, x, k):
    """Bank (dword address mod 32) of lane's lookup k of word x in the DMA kernel's slice tables."""
    h = (lane >> 3) & 3
    return (v_perm(x, (lane & 7) * 4 + 32 * (k ^ h), 0x0C0C0400 + ((k ^ h) << 8)) // 4) % 32


def merge_shift(lds, m, s):
    r = 0
    for t in range(8):
        sh = (s >> (4 * t - 2)) if 4 * t >= 2 else ((s << 2) & 0xFFFFFFFF)
        r ^= int(lds[((sh & 0x3C) | (hole(MERGE_HOLE + 4 * m + (t >> 1)) + 64 * (t & 1))) // 4])
    return r


def model_dma_item(lds, mem: bytes, base: int, stride: int, flen: int, n: int, f: int, garbage: bytes,
                   chains=DMA_CHAINS):
    """The four FCS values fcs_dma_kernel computes for the wave item whose first frame is f (frames
    >= n are None). mem is the whole arena, base its frame-0 offset; bytes a window reads outside
    the slot image come from `garbage` (they must all be masked)."""
    lo16 = (base & ~3) & ~15
    hi16 = (((base + (n - 1) * stride + flen + 3) & ~3) + 15) & ~15
    smax = hi16 - DMA_SLOT
    S = base + f * stride
    src = min(max(S & ~15, lo16), smax)
    img = bytearray(garbage[:64]) + bytearray(DMA_SLOT) + bytearray(garbage[64:128])
    chunk = mem[src:src + DMA_SLOT]
    img[64:64 + len(chunk)] = chunk
    zmax = max(4, DMA_COVER - flen)
    cl = 24 // chains
    out = []
    for g in range(4):
        regs = []
        for c in range(16):
            lane = 16 * g + c
            ec = dma_end_off(c)
            x = (S - src) + g * stride + flen - ec - CHUNK
            r = x & 3
            a = 64 + (x & ~3)
            d = [int.from_bytes(img[a + 4 * q:a + 4 * q + 4], "little") for q in range(25)]
            w = [alignbyte(d[i + 1], d[i], r) for i in range(24)]
            zc = (DMA_COVER - flen) if c == 15 else (4 if dma_short_lane(c) else 0)
            for i in range(8):
                if 4 * i < zmax:
                    t = max(0, min(4, zc - 4 * i))
                    w[i] &= (0xFFFFFFFFFFFFFFFF << (8 * t)) & 0xFFFFFFFF
            x0 = int(lds[(hole(INV_HOLE + zc // 32) + (zc % 32) * 4) // 4]) if c == 15 else 0
            xs = [w[h * cl] ^ (x0 if h == 0 else 0) for h in range(chains)]
            for i in range(cl):
                for h in range(chains):
                    xs[h] = step4_l8(lds, xs[h], lane) ^ (w[h * cl + i + 1] if i < cl - 1 else 0)
            m = xs[chains - 1]
            for h in range(chains - 1):
                m = merge_shift(lds, chains - 2 - h, xs[h]) ^ m
            lanebase = 128 + (lane & 31) * 4
            s = 0
            for t in range(8):
                sh = (m >> (4 * t - 8)) if 4 * t >= 8 else ((m << (8 - 4 * t)) & 0xFFFFFFFF)
                s ^= int(lds[(((sh & 0xF00) | lanebase) + t * 4096) // 4])
            regs.append(s)
        v = 0
        for s in regs:
            v ^= s
        out.append((~v & 0xFFFFFFFF) if f + g < n else None)
    return out


# ---- fcs_segil_kernel: frame-interleaved segments ----
def model_segil_window_value(lds, win: bytes, lane: int, z: int, x0: int, chains=DMA_CHAINS):
    """One lane window of fcs_segil_kernel (as fcs_dma_kernel's): 96 bytes, the first z masked,
    x0 XORed into chain 0's start; two chains merged, shifted by the lane table A_{e_c}."""
    cl = 24 // chains
    w = [int.from_bytes(win[4 * i:4 * i + 4], "little") for i in range(24)]
    for i in range(24):
        t = max(0, min(4, z - 4 * i))
        w[i] &= (0xFFFFFFFFFFFFFFFF << (8 * t)) & 0xFFFFFFFF
    xs = [w[h * cl] ^ (x0 if h == 0 else 0) for h in range(chains)]
    for i in range(cl):
        for h in range(chains):
            xs[h] = step4_l8(lds, xs[h], lane) ^ (w[h * cl + i + 1] if i < cl - 1 else 0)
    m = xs[chains - 1]
    for h in range(chains - 1):
        m = merge_shift(lds, chains - 2 - h, xs[h]) ^ m
    lanebase = 128 + (lane & 31) * 4
    s = 0
    for t in range(8):
        sh = (m >> (4 * t - 8)) if 4 * t >= 8 else ((m << (8 - 4 * t)) & 0xFFFFFFFF)
        s ^= int(lds[(((sh & 0xF00) | lanebase) + t * 4096) // 4])
    return s


def model_segil_frame(lds, frame: bytes, garbage: bytes):
    """FCS of one frame by fcs_segil_kernel's decomposition: a front segment of Lf = L - 1524 (m - 1)
    bytes, then 1524-B segments. Each segment is a 1524-B cover of 16 lane windows ending at the
    segment end. Front: lane c masks the zr = (1524 - Lf) - ws_c bytes of its window before the frame
    start (whole window: dropped), short lanes at least their 4-byte overlap, and the lane holding
    the first byte unmasked starts from INV[zr]. Other segments: only the short lanes' overlap word;
    lane 15 starts from the frame's CRC state after the previous segment (the row XOR)."""
    L = len(frame)
    m = -(-L // DMA_COVER)
    lf = L - DMA_COVER * (m - 1)
    padded = bytes(garbage[:DMA_COVER]) + frame
    acc = 0
    for r in range(m):
        end = DMA_COVER + lf + DMA_COVER * r
        cover = padded[end - DMA_COVER:end]
        v = 0
        for c in range(16):
            ws = DMA_COVER - dma_end_off(c) - CHUNK
            win = cover[ws:ws + CHUNK]
            short = 4 if dma_short_lane(c) else 0
            if r == 0:
                zr = (DMA_COVER - lf) - ws
                if zr >= CHUNK:
                    continue
                z = max(max(zr, 0), short)
                x0 = int(lds[(hole(INV_HOLE + zr // 32) + (zr % 32) * 4) // 4]) if (zr >= 0 and z == zr) else 0
            else:
                z = short
                x0 = acc if c == 15 else 0
            v ^= model_segil_window_value(lds, win, c, z, x0)
        acc = v
    return ~acc & 0xFFFFFFFF


# ---- fcs_wide_kernel: 128-B windows at e_c = 124 c, 8 KiB slots (fcs_tables.hpp kWide*) ----
BLOB_STREAM = BLOB_MERGE + 11 * 8 * 16
BLOB_STREAM_K1 = BLOB_STREAM + (24 + 17 + 4) * 128
BLOB_LANE_WIDE = BLOB_STREAM_K1 + 64
BLOB_LANE_WIDE26 = BLOB_LANE_WIDE + 8 * 16 * 32
BLOB_LANE_WIDE30 = BLOB_LANE_WIDE26 + 8 * 16 * 32
BLOB_INV_WIDE = BLOB_LANE_WIDE30 + 8 * 16 * 32
WIDE_WIN, WIDE_SLOT = 128, 8192
WIDE_COVER = 124 * 15 + WIDE_WIN   # 1988
WIDE_MERGE_HOLE, WIDE_INV_HOLE = 128, 132
WIDE_MID = [wd for wd in range(15, 25) if (wd - 1) % 4]   # mid-length widths (fcs_tables.hpp wide_mid_ok)
BLOB_LANE_MID = BLOB_INV_WIDE + WIDE_WIN                  # kBlobLaneMid: one [8][16][32] set per WD 15..24
WIDE8 = [wd for wd in range(11, 29) if (wd - 1) % 4]    # eight-lane group widths (fcs_tables.hpp wide8_ok)
BLOB_LANE8 = BLOB_LANE_MID + (24 - WIDE_MID[0] + 1) * 4096   # kBlobLane8: one set per WD 11..28
WIDE4 = [wd for wd in range(9, 27) if (wd - 1) % 16]     # four-lane group widths (fcs_tables.hpp wide4_ok)
BLOB_LANE4 = BLOB_LANE8 + (28 - 11 + 1) * 4096            # kBlobLane4: one set per WD 9..26
WIDE_CL0 = {**{wd: wd - 2 * (wd // 4) for wd in WIDE_MID + WIDE8 + WIDE4}, 32: 16, 30: 14, 26: 12}   # chain 0's words


def wide_end_off(c, wd=32):
    return (4 * wd - 4) * c


def wide_slot(wd):
    return 8192 if wd == 32 else (7168 if wd > 24 else 6144)


def wide_cover(wd):
    return 15 * (4 * wd - 4) + 4 * wd


def wide8_cover(wd):
    return 7 * (4 * wd - 4) + 4 * wd


def wide4_cover(wd):
    return 3 * (4 * wd - 4) + 4 * wd


def wide4_wd(flen):
    """The width the host picks for a four-lane-group frame (fcs_launch.hpp wide4_wd)."""
    return next(wd for wd in WIDE4 if wide4_cover(wd) >= flen)


def wide8_wd(flen):
    """The width the host picks for an eight-lane-group frame (fcs_launch.hpp wide8_wd)."""
    return next(wd for wd in WIDE8 if wide8_cover(wd) >= flen)


def wide_mid_wd(flen):
    """The width the host picks for a mid-length frame (fcs_launch.hpp wide_mid_wd)."""
    return next(wd for wd in WIDE_MID if wide_cover(wd) >= flen)


def build_lds_wide(blob, wd=32, G=16):
    """fcs_wide_kernel<WD>'s 64 KiB table image: the slice tables as fcs_dma_kernel's; holes 16t+n
    the lane tables A_{(4 WD - 4) c}; holes 128..131 the chain merge A_{4 (WD - CL0)}; holes
    132..135 INV[0..127]."""
    lane_blob = {32: BLOB_LANE_WIDE, 30: BLOB_LANE_WIDE30, 26: BLOB_LANE_WIDE26}.get(wd)
    if G == 4:
        lane_blob = BLOB_LANE4 + (wd - 9) * 4096
    elif G == 8:
        lane_blob = BLOB_LANE8 + (wd - 11) * 4096
    elif lane_blob is None:
        lane_blob = BLOB_LANE_MID + (wd - WIDE_MID[0]) * 4096
    k = (4 * (wd - WIDE_CL0[wd])) // 8
    lds = np.zeros(65536 // 4, dtype=np.uint32)
    for e in range(256):
        for sl in range(4):
            lds[(e * 256 + sl * 32) // 4:(e * 256 + sl * 32) // 4 + 8] = blob[BLOB_SLICE + 256 * (3 - sl) + e]
    for i in range(4096):
        lds[(hole(i >> 5) + (i & 31) * 4) // 4] = blob[lane_blob + i]
    for t in range(8):
        for e in range(16):
            lds[(hole(WIDE_MERGE_HOLE + (t >> 1)) + 64 * (t & 1) + 4 * e) // 4] = blob[BLOB_MERGE + (k - 1) * 128 + t * 16 + e]
    for z in range(WIDE_WIN):
        lds[(hole(WIDE_INV_HOLE + z // 32) + (z % 32) * 4) // 4] = blob[BLOB_INV_WIDE + z]
    return lds


def wide_front(flen, wd=32, G=16):
    """Front lane cf (the last lane whose window reaches into the frame) and its leading bytes zc."""
    step = 4 * wd - 4
    cf = min(G - 1, (flen - 1) // step)
    return cf, step * cf + 4 * wd - flen


def model_wide_item(lds, mem: bytes, base: int, stride: int, flen: int, n: int, f: int, garbage: bytes, wd=32, G=16):
    """The four FCS values fcs_wide_kernel computes for the wave item whose first frame is f: lanes
    c <= cf are live; each masks its first word (its neighbour's last) except the front lane, which
    masks its zc leading bytes and starts from INV[zc]; two 16-word chains merged with A_64; lane
    shift A_{124 c}. Bytes a window reads outside the slot come from `garbage` (all masked)."""
    lo16 = (base & ~3) & ~15
    hi16 = (((base + (n - 1) * stride + flen + 3) & ~3) + 15) & ~15
    slot = wide_slot(wd)
    win, cl0 = 4 * wd, WIDE_CL0[wd]
    smax = hi16 - slot
    S = base + f * stride
    src = min(max(S & ~15, lo16), smax)
    pad = 2048
    img = bytearray(garbage[:pad]) + bytearray(slot) + bytearray(garbage[pad:pad + 64])
    chunk = mem[src:src + slot]
    img[pad:pad + len(chunk)] = chunk
    cf, zc = wide_front(flen, wd, G)
    out = []
    for g in range(64 // G):
        v = 0
        for c in range(cf + 1):
            lane = G * g + c
            x = (S - src) + g * stride + flen - wide_end_off(c, wd) - win
            r = x & 3
            a = pad + (x & ~3)
            d = [int.from_bytes(img[a + 4 * q:a + 4 * q + 4], "little") for q in range(wd + 1)]
            w = [alignbyte(d[i + 1], d[i], r) for i in range(wd)]
            z = zc if c == cf else 4
            for i in range(wd):
                t = max(0, min(4, z - 4 * i))
                w[i] &= (0xFFFFFFFFFFFFFFFF << (8 * t)) & 0xFFFFFFFF
            x0 = int(lds[(hole(WIDE_INV_HOLE + zc // 32) + (zc % 32) * 4) // 4]) if c == cf else 0
            xs = [w[0] ^ x0, w[cl0]]
            for i in range(cl0):
                xs[0] = step4_l8(lds, xs[0], lane) ^ (w[i + 1] if i < cl0 - 1 else 0)
            for i in range(wd - cl0):
                xs[1] = step4_l8(lds, xs[1], lane) ^ (w[cl0 + i + 1] if i < wd - cl0 - 1 else 0)
            m = merge_shift(lds, 0, xs[0]) ^ xs[1]   # A_64 at the merge holes (WIDE_MERGE_HOLE == MERGE_HOLE)
            lanebase = 128 + (lane & 31) * 4
            s = 0
            for t in range(8):
                sh = (m >> (4 * t - 8)) if 4 * t >= 8 else ((m << (8 - 4 * t)) & 0xFFFFFFFF)
                s ^= int(lds[(((sh & 0xF00) | lanebase) + t * 4096) // 4])
            v ^= s
        out.append((~v & 0xFFFFFFFF) if f + g < n else None)
    return out



# ---- fcs_segw_kernel<WD>: frame-interleaved segments of the wide kernel's cover (WD 26 / 30) ----
def model_wide_window_value(lds, win: bytes, lane: int, z: int, x0: int, wd: int):
    """One lane window of fcs_wide_kernel<WD> (4 WD bytes, the first z masked, x0 into chain 0's
    start): two chains merged with A_{4 (WD - CL0)}, lane shift A_{(4 WD - 4) c}."""
    cl0 = WIDE_CL0[wd]
    w = [int.from_bytes(win[4 * i:4 * i + 4], "little") for i in range(wd)]
    for i in range(wd):
        t = max(0, min(4, z - 4 * i))
        w[i] &= (0xFFFFFFFFFFFFFFFF << (8 * t)) & 0xFFFFFFFF
    xs = [w[0] ^ x0, w[cl0]]
    for i in range(cl0):
        xs[0] = step4_l8(lds, xs[0], lane) ^ (w[i + 1] if i < cl0 - 1 else 0)
    for i in range(wd - cl0):
        xs[1] = step4_l8(lds, xs[1], lane) ^ (w[cl0 + i + 1] if i < wd - cl0 - 1 else 0)
    m = merge_shift(lds, 0, xs[0]) ^ xs[1]
    lanebase = 128 + (lane & 31) * 4
    s = 0
    for t in range(8):
        sh = (m >> (4 * t - 8)) if 4 * t >= 8 else ((m << (8 - 4 * t)) & 0xFFFFFFFF)
        s ^= int(lds[(((sh & 0xF00) | lanebase) + t * 4096) // 4])
    return s


def model_segw_frame(lds, frame: bytes, garbage: bytes, wd: int):
    """FCS of one frame by fcs_segw_kernel<WD>'s decomposition: a front segment of
    Lf = L - C (m - 1) bytes (C = wide_cover(WD)), then C-byte segments, each the wide kernel's 16
    windows ending at the segment end. Front: the wide kernel's front lane cf and zc for length Lf
    (INV[zc], lanes past cf dropped). Other segments: every lane masks its first word (the next
    lane's last) except lane 15, whose window starts at the segment start and whose chain starts
    from the frame's CRC state after the previous segment."""
    C = wide_cover(wd)
    step, win = 4 * wd - 4, 4 * wd
    L = len(frame)
    m = -(-L // C)
    lf = L - C * (m - 1)
    padded = bytes(garbage[:C]) + frame
    acc = 0
    for r in range(m):
        end = C + lf + C * r
        v = 0
        for c in range(16):
            ws = end - step * c - win
            w = padded[ws:ws + win]
            if r == 0:
                cf, zc = wide_front(lf, wd)
                if c > cf:
                    continue
                z = zc if c == cf else 4
                x0 = int(lds[(hole(WIDE_INV_HOLE + zc // 32) + (zc % 32) * 4) // 4]) if c == cf else 0
            else:
                z = 0 if c == 15 else 4
                x0 = acc if c == 15 else 0
            v ^= model_wide_window_value(lds, w, c, z, x0, wd)
        acc = v
    return ~acc & 0xFFFFFFFF


# ---- inet_stream_kernel: a packed 64-packet window summed from 6 KiB slot items ----
def _dot4(x, w, c):
    """v_dot4_u32_u8: c + sum of the four byte products of x and w."""
    return c + sum(((x >> (8 * k)) & 0xFF) * ((w >> (8 * k)) & 0xFF) for k in range(4))


def model_inet_window(span: bytes, starts, total: int, slot=6144, lane_bytes=96):
    """Per-packet sums E + 256 O (even- and odd-addressed bytes of each packet, span positions
    relative to the 16-B aligned span start) as inet_stream_kernel attributes them: items of `slot`
    bytes, lane l takes bytes [96 l, 96 l + 96) of an item piece by piece; the packet holding the
    lane's first byte by binary search over the 64 starts (inactive lanes hold `total`); a piece
    holds at most one packet start, split by the running dot4 sums before its dword plus that
    dword's bytes below it; the span's first and last pieces are masked to [starts[0], total)."""
    st = list(starts) + [total] * (64 - len(starts))
    acc = [0] * 64
    st0 = st[0]
    for k in range(-(-total // slot)):
        for lane in range(slot // lane_bytes):
            P0 = k * slot + lane_bytes * lane
            if P0 >= total:
                continue
            cur = 0
            b = 32
            while b:
                if st[cur + b] <= P0:
                    cur += b
                b >>= 1
            nxt = st[cur + 1] if cur + 1 < 64 else total
            E = O = 0
            for q in range(lane_bytes // 16):
                Pq = P0 + 16 * q
                if Pq >= total:
                    break
                piece = bytearray(span[Pq:Pq + 16].ljust(16, b"\0"))
                if Pq < st0 or total - Pq < 16:
                    lo = st0 - Pq if Pq < st0 else 0
                    hi = min(16, total - Pq)
                    for j in range(16):
                        if not lo <= j < hi:
                            piece[j] = 0
                x = [int.from_bytes(piece[4 * d:4 * d + 4], "little") for d in range(4)]
                if nxt <= Pq:
                    acc[cur] += E + (O << 8)
                    E = O = 0
                    cur += 1
                    nxt = st[cur + 1] if cur + 1 < 64 else total
                e, o = [0] * 4, [0] * 4
                ce = co = 0
                for d in range(4):
                    ce = _dot4(x[d], 0x00010001, ce)
                    co = _dot4(x[d], 0x01000100, co)
                    e[d], o[d] = ce, co
                bnd = nxt - Pq
                if bnd < min(16, total - Pq):
                    db, lm = bnd >> 2, (1 << (8 * (bnd & 3))) - 1
                    eb = 0 if db == 0 else e[db - 1]
                    ob = 0 if db == 0 else o[db - 1]
                    eb = _dot4(x[db], 0x00010001 & lm, eb)
                    ob = _dot4(x[db], 0x01000100 & lm, ob)
                    acc[cur] += (E + eb) + ((O + ob) << 8)
                    cur += 1
                    nxt = st[cur + 1] if cur + 1 < 64 else total
                    E, O = e[3] - eb, o[3] - ob
                else:
                    E += e[3]
                    O += o[3]
            acc[cur] += E + (O << 8)
    return acc
