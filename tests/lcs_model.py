"""CPU model of the lane-chunk carry decomposition of packed variable-length FCS batches
(TEST INFRASTRUCTURE; round 4, the successor of tests/stream_model.py's per-chunk decomposition).

The reference computes one FCS per frame (/root/reference/src/ether_fcs.c:4-19); this module
states, in plain Python, how a wave of 64 lanes can compute the FCSs of a packed run of frames
(offs[i + 1] == offs[i] + lens[i], 64 <= len <= 1536) so that per lane only ONE table shift per
G x 64 bytes is needed, and checks it against zlib in tests/test_lcs_model.py. It is never used
to produce product results.

Notation as stream_model.py: R(s, M) is the CRC register after bytes M from register s (reflected,
poly 0xEDB88320, no complements); A_n advances a register over n zero bytes (linear, invertible);
the reference FCS of a frame B is ~R(~0, B).

Layout. A unit's bytes are walked from X0 (the 16-B boundary at or below its first frame) in items
of 64 lane-chunks of G sub-chunks of 64 bytes: lane l of item t owns the lane-chunk
C = X0 + 64 G (64 t + l), i.e. the lane-chunks of all items form one linear sequence. A sub-chunk
holds at most one frame boundary (frames >= 64 B).

The lane's chain runs over its whole lane-chunk from register 0, word by word (x <- A_4(x ^ w)),
and is RESET at a boundary p = 4 k + r inside a sub-chunk (word k, byte r) instead of tapped and
shifted: before word k the lane saves its state s_k; the frame ending at p gets the end tap
T = A_4(s_k ^ (w_k & the r bytes before p)) = A_{4-r}(R(s_k, those bytes)), and the chain goes on
from INV_r ^ (w_k & the bytes from p on), INV_r = A_{-r}(~0) (r zero bytes take it to ~0), i.e.
exactly as if the frame starting at p had started from ~0. So:

- the lane-chunk's final state x_end is, if the lane-chunk holds a boundary, the full register of
  the frame holding its last byte (the "tail frame"), and otherwise its bytes' contribution
  R(0, C);
- a frame that starts and ends in one lane-chunk has T_e = A_{4-r_e}(R(~0, frame)) directly;
- a frame spanning lane-chunks a < ... < b (it starts in a, ends in b): every lane m in [a, b)
  adds A_{64 G (b - 1 - m)}(x_end(m)) to the frame's accumulator S (one shift per lane-chunk, by
  a whole number of lane-chunks), and then, with the end at word k_e of sub-chunk s_e of b,

      A_{4 - r_e}(R(~0, frame)) = A_{64 s_e}( A_{4 (k_e + 1)}(S) ) ^ T_e,

which holds for frames inside one lane-chunk too with S = 0. The close therefore takes per frame
two forward shifts, the end tap, and A_{-(4 - r_e)}.
"""
import zlib

from stream_model import T0, zstep, word_step

CH = 64


def fcs_zlib(b: bytes) -> int:
    return zlib.crc32(b) & 0xFFFFFFFF


def _inv(r):
    """INV_r = A_{-r}(~0)."""
    return zstep(0xFFFFFFFF, -r)


def model_lcs(arena: bytes, offs, lens, G=4, unit_frames=None, counts=None):
    n = len(offs)
    out = [None] * n
    ranges = [(0, n)] if not unit_frames else [(i, min(n, i + unit_frames)) for i in range(0, n, unit_frames)]
    for f0, f1 in ranges:
        _unit(arena, offs, lens, f0, f1, out, G, counts)
    return out


def _unit(arena, offs, lens, f0, f1, out, G, counts):
    LC = CH * G                       # lane-chunk bytes
    s0 = offs[f0]
    X0 = s0 & ~15
    E = offs[f1 - 1] + lens[f1 - 1]   # the unit's end
    padded = bytes(arena) + bytes(64 * LC + 16)
    # boundaries: the unit's first start, every frame end (the last one is the unit end)
    ends = {offs[i] + lens[i]: i for i in range(f0, f1)}
    nlc = (E - X0 + LC - 1) // LC     # lane-chunks of the unit (rounded up to whole items in the kernel)
    acc = {i: 0 for i in range(f0, f1)}
    tap = {}
    for c in range(nlc):
        C = X0 + LC * c
        x = 0                          # chain state before the next word
        for s in range(G):
            a = C + CH * s
            bps = [p for p in range(a, a + CH) if p in ends or p == s0]
            assert len(bps) <= 1, "two boundaries in one sub-chunk"
            k = r = None
            if bps:
                p = bps[0]
                k, r = (p - a) >> 2, (p - a) & 3
            for i in range(16):
                w = int.from_bytes(padded[a + 4 * i:a + 4 * i + 4], "little")
                if i == k:
                    lo = w & ((1 << (8 * r)) - 1)
                    hi = w ^ lo
                    if p in ends:
                        tap[ends[p]] = word_step(x, lo)
                    x = word_step(_inv(r), hi) if p < E else 0   # reset (nothing follows the unit end)
                else:
                    x = word_step(x, w)
        x_end = x
        # the lane-chunk's last byte and the frame holding it (the tail frame), if any
        q = C + LC - 1
        if q < s0 or C >= E:
            continue
        o = _frame_at(offs, lens, f0, f1, min(q, E - 1))
        if q >= E:
            continue                  # the unit ends in this lane-chunk: its tail is nothing
        e = offs[o] + lens[o]
        b = (e - X0) // LC            # lane-chunk holding the end (e == its start: tap 0 there)
        j = b - c - 1
        assert j >= 0
        acc[o] ^= zstep(x_end, LC * j)
        if counts is not None:
            counts["shifts"] = counts.get("shifts", 0) + 1
    for i in range(f0, f1):
        e = offs[i] + lens[i]
        rel = e - X0
        b = rel // LC
        within = rel - LC * b
        s_e, k_e, r_e = within // CH, (within % CH) >> 2, within & 3
        # an end on a lane-chunk edge has no tap when nothing follows it (the unit's end): T_e = 0
        assert i in tap or within == 0
        v = zstep(zstep(acc[i], 4 * (k_e + 1)), CH * s_e) ^ tap.get(i, 0)
        reg = zstep(v, -(4 - r_e))
        out[i] = ~reg & 0xFFFFFFFF


def _frame_at(offs, lens, f0, f1, q):
    lo, hi = f0, f1 - 1
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if offs[mid] <= q:
            lo = mid
        else:
            hi = mid - 1
    return lo
