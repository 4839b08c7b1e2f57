"""CPU model of the arena-stream decomposition of variable-length FCS batches (TEST INFRASTRUCTURE).

SURVEY.md §7 / VERDICT r2 item 2: instead of dealing frame-anchored 96-B chunks to the lanes
(fcs_flat_kernel), stream the packed arena in 64-B chunks at fixed, 16-B-aligned positions (so an
item of 64 chunks is one coalesced 4 KiB LDS-DMA, independent of any dealing) and handle frame
boundaries with taps and a per-frame combine. This module states that decomposition in plain
Python, checks it against zlib (= the reference ether_fcs, /root/reference/src/ether_fcs.c:4-19)
in tests/test_stream_model.py, and counts the work per item for the comparison with the flat
kernel's dealing. It is never used to produce product results.

Notation: R(s, M) is the CRC register after bytes M from register s (reflected, poly 0xEDB88320,
no complements); A_n is "advance over n zero bytes" (linear, invertible); for a frame B = [s, e)
of the arena the reference FCS is ~R(~0, B) = ~(A_len(~0) ^ R(0, B)).

Chunk l of an item covers [a_l, a_l + 64); its chain L_l = R(0, chunk bytes) runs from register 0
over all 64 bytes whatever frames they belong to. For a boundary p in chunk l (a frame start, or
the batch's last frame end), the lane takes a TAP of its chain: k = (p - a_l) >> 2, r = (p - a_l)
& 3, s_k the chain after k words, and T'(p) = A_4(s_k ^ (w_k & low r bytes)) = A_{4-r}(R(0,[a_l, p))).
With these, for a frame B whose start s lies in chunk ls and whose end e in chunk le (> ls, since
every frame is at least 64 B long):

    R(~0, B) = A_{r_e - 4}( T'(e) ^ A_{4 (k_e + 1)}( acc_B ) ),
    acc_B    = XOR_{m = ls .. le-1} A_{64 (le - m - 1)}( V_m ),
    V_m      = L_m                                          (m > ls)
    V_ls     = L_ls ^ A_{4 (15 - k_s)}(T'(s)) ^ A_{64 - sigma_s}(~0)

i.e. every chunk goes to the frame that holds its last byte, shifted by whole chunks to the chunk
holding that frame's end; the chunk where a frame starts adds the frame's all-ones start as it
would stand at the chunk end (the tap removes the previous frame's bytes); the frame's end tap
closes it. The only per-lane work beyond the chain is one tap (frames >= 64 B put at most one
boundary in a 64-B chunk), one shift by a multiple of 4 bytes at a start, and one chunk shift;
per frame, two shifts at the end.
"""
import numpy as np

POLY = 0xEDB88320
CH = 64            # chunk bytes per lane
ITEM = 64 * CH     # bytes per item (one 4 KiB DMA)


def _tables():
    t0 = []
    for b in range(256):
        r = b
        for _ in range(8):
            r = (r >> 1) ^ (POLY if r & 1 else 0)
        t0.append(r)
    inv = [0] * 256
    for b in range(256):
        inv[t0[b] >> 24] = b
    return t0, inv


T0, TOPINV = _tables()


def zstep(s, n=1):
    """A_n(s) for n >= 0 (zero bytes) or the inverse for n < 0."""
    for _ in range(n):
        s = (s >> 8) ^ T0[s & 0xFF]
    for _ in range(-n):
        i = TOPINV[s >> 24]
        s = ((s ^ T0[i]) << 8 & 0xFFFFFFFF) | i
    return s


def step_byte(s, b):
    return (s >> 8) ^ T0[(s ^ b) & 0xFF]


def word_step(s, w):
    """A_4(s ^ w): the slice-by-4 step the kernels evaluate with four table lookups."""
    return zstep(s ^ w, 4)


def chain(words):
    """The lane chain: states s_0 = 0, s_{i+1} = A_4(s_i ^ w_i); returns all 17 states."""
    st = [0]
    for w in words:
        st.append(word_step(st[-1], w))
    return st


def fcs_ref(b: bytes):
    s = 0xFFFFFFFF
    for x in b:
        s = step_byte(s, x)
    return ~s & 0xFFFFFFFF


class Counts:
    """Work of the decomposition, counted per item (wave-instruction granularity)."""

    def __init__(self):
        self.items = 0
        self.item_overlap = 0       # items a wave loads that a neighbouring range loads too
        self.frames = 0
        self.bytes = 0
        self.boundaries = 0
        self.lanes_with_boundary = 0


def model_stream(arena: bytes, offs, lens, unit_frames=None, counts: Counts = None):
    """FCS of packed frames (offs[i+1] == offs[i] + lens[i], 64 <= len <= 1536) by the arena-stream
    decomposition. `unit_frames`: split the batch into ranges of this many frames processed
    independently (a wave's dispenser chunks: each range starts its own item sequence at the
    128-B line below its first frame, so the lines at range edges are loaded twice)."""
    n = len(offs)
    out = [None] * n
    ranges = [(0, n)] if not unit_frames else [(i, min(n, i + unit_frames)) for i in range(0, n, unit_frames)]
    for f0, f1 in ranges:
        _model_range(arena, offs, lens, f0, f1, out, counts)
    return out


def _model_range(arena, offs, lens, f0, f1, out, counts):
    s0 = offs[f0]
    e_last = offs[f1 - 1] + lens[f1 - 1]
    X0 = s0 & ~127                      # the range's first item starts at the 128-B line below
    starts = {offs[i]: i for i in range(f0, f1)}          # boundary position -> frame starting there
    end_of = {offs[i] + lens[i]: i for i in range(f0, f1)}  # boundary position -> frame ending there
    acc = {i: 0 for i in range(f0, f1)}
    endtap = {}
    nitems = (e_last - X0 + ITEM - 1) // ITEM
    padded = bytes(arena) + bytes(ITEM + 16)
    for t in range(nitems):
        X = X0 + ITEM * t
        if counts:
            counts.items += 1
        bset = set()
        for l in range(64):
            a = X + CH * l
            words = [int.from_bytes(padded[a + 4 * q:a + 4 * q + 4], "little") for q in range(CH // 4)]
            st = chain(words)
            L = st[-1]
            # the boundary in this chunk, if any (frames >= 64 B: at most one)
            bps = [p for p in range(a, a + CH) if p in starts or p in end_of]
            assert len(bps) <= 1, "two boundaries in one chunk: a frame shorter than the chunk"
            V = L
            if bps:
                p = bps[0]
                sig = p - a
                k, r = sig >> 2, sig & 3
                wk = words[k] if k < len(words) else 0
                Tp = word_step(st[k], wk & ((1 << (8 * r)) - 1))
                bset.add(p)
                if counts:
                    counts.lanes_with_boundary += 1
                if p in end_of:                        # closes the frame ending here
                    endtap[end_of[p]] = (Tp, k, r)
                if p in starts:                        # opens the frame starting here
                    V = L ^ zstep(Tp, 4 * (15 - k)) ^ zstep(0xFFFFFFFF, CH - sig)
            # the frame holding the chunk's last byte
            q = a + CH - 1
            o = _frame_at(offs, lens, f0, f1, q)
            if o is None:
                continue
            e = offs[o] + lens[o]
            le = (e - X0) // CH
            m = (a - X0) // CH
            j = le - m - 1
            assert 0 <= j <= 24
            acc[o] ^= zstep(V, CH * j)
        if counts:
            counts.boundaries += len(bset)
    for i in range(f0, f1):
        Tp, k, r = endtap[i]
        reg = zstep(Tp ^ zstep(acc[i], 4 * (k + 1)), r - 4)
        out[i] = ~reg & 0xFFFFFFFF
        if counts:
            counts.frames += 1
            counts.bytes += lens[i]


def _frame_at(offs, lens, f0, f1, q):
    """Index of the frame of [f0, f1) holding byte q, or None (bytes before or after the range)."""
    if q < offs[f0] or q >= offs[f1 - 1] + lens[f1 - 1]:
        return None
    lo, hi = f0, f1 - 1
    while lo < hi:                       # last frame whose start is <= q
        mid = (lo + hi + 1) // 2
        if offs[mid] <= q:
            lo = mid
        else:
            hi = mid - 1
    return lo


def imix_structure(lens, unit_frames, base=0):
    """Structural work of both decompositions on one packed stream, without computing CRCs:
    items, chunks, boundaries and overlap of the arena stream (64-B chunks, 4 KiB items, ranges of
    unit_frames frames) against the flat kernel's frame-anchored 96-B chunks dealt 64 per item."""
    lens = np.asarray(lens, dtype=np.int64)
    offs = base + np.concatenate([[0], np.cumsum(lens)[:-1]])
    total = int(lens.sum())
    # arena stream
    items = 0
    for f0 in range(0, len(lens), unit_frames):
        f1 = min(len(lens), f0 + unit_frames)
        X0 = max(int(offs[f0]) & ~127, base & ~15)
        e = int(offs[f1 - 1] + lens[f1 - 1])
        items += (e - X0 + ITEM - 1) // ITEM
    # flat kernel: ceil(len / 96) chunks per frame, dealt 64 at a time per 64-frame window
    k = (lens + 95) // 96
    flat_items = 0
    for w in range(0, len(lens), 64):
        flat_items += int((k[w:w + 64].sum() + 63) // 64)
    return {"bytes": total, "frames": len(lens),
            "stream_items": items, "stream_bytes_per_item": total / items,
            "stream_chunk_bytes": CH, "stream_lane_utilisation": total / (items * ITEM),
            "stream_boundaries_per_item": (len(lens) + 1) / items,
            "flat_items": flat_items, "flat_bytes_per_item": total / flat_items,
            "flat_lane_utilisation": total / (flat_items * 64 * 96)}
