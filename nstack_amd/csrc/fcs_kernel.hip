// fcs_kernel.hip — batched Ethernet FCS (CRC-32/ISO-HDLC) for CDNA4 / gfx950 (MI355X).
//
// Replaces the per-frame byte loop of ether_fcs() (/root/reference/src/ether_fcs.c:13-16) with
// one launch over many independent frames. Result per frame is bit-identical to ether_fcs().
//
// Work decomposition:
//   * one QUARTER-WAVE (16 lanes) per frame; lane j owns the 96-byte chunk that ends 96*j bytes
//     before the frame end, so 16 lanes cover one 1536-byte "segment"; longer frames are walked
//     segment by segment, front to back (jumbo 9000 B = 6 segments); a wave works on 4 frames;
//   * each lane loads its chunk with 6 x global_load_dwordx4 + 1 dword from a 4-byte aligned
//     address (this layout streams HBM at the rate of a coalesced read: tools/microbench), two
//     chunks in flight per lane; the words are re-aligned to the frame end with v_alignbyte_b32
//     and the bytes in front of the frame start are zeroed;
//   * the lane runs its 24 words as four independent 6-word slice-by-4 chains (ILP 4): per word
//     4 ds_read_b32 from byte tables replicated 32x in LDS (replica = lane & 31 -> every 32-lane
//     LDS access is bank-conflict free), each address formed by ONE v_perm_b32; the chains are
//     merged as A_48(A_24(a) ^ b) ^ (A_24(c) ^ d) with nibble tables;
//   * the frame's all-ones initial register is injected as the front lane's start value
//     INV[z] = A_z^{-1}(~0) (z = zero bytes in front of the frame start); across segments a
//     lane accumulates S = A_1536(S) ^ segment value, so consecutive items stay independent;
//   * at the frame end lane j shifts its register by 96*j zero bytes (per-lane nibble tables,
//     bank = lane), the 16 registers are XOR-reduced with 4 DPP steps and lane 15 stores ~crc.
// No MFMA: a byte-stream codec bounded by HBM read bandwidth (roofline: DESIGN.md §4).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fcs_launch.hpp"
#include "fcs_tables.hpp"
#include "wave_sync.hpp"

namespace fcs {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Frame slots (quarter-waves) per workgroup of NT threads; LDS (150 KiB) -> 1 WG per CU.
template <int NT> constexpr int kSlotsPerWg = NT / kGroup;

constexpr int kSingleMaskWords = kSingleMaxLead / 4;   // SINGLE variant: front-lane masks for words < 8
#ifndef FCS_CHAINS
#define FCS_CHAINS 2                               // independent chains per lane (2 or 4)
#endif

// Loads through address space 1 (global): flat loads would also count on lgkmcnt and make every
// LDS wait drain the prefetched chunk loads.
template <typename T>
__device__ __forceinline__ T gload(uint64_t addr) {
#ifdef FCS_NT   // measurement-only build: non-temporal (nt) frame loads
    return __builtin_nontemporal_load(reinterpret_cast<const __attribute__((address_space(1))) T *>(addr));
#else
    return *reinterpret_cast<const __attribute__((address_space(1))) T *>(addr);
#endif
}

// a ^ b ^ c in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Clears the low t bits of w, t clamped to 0..32 (bytes of a window before the frame start). The
// clamp is one v_med3_i32: written as min/max the compiler proves t >= 0 after the max, turns the
// min unsigned and keeps two instructions.
__device__ __forceinline__ uint32_t clear_low_bits(uint32_t w, int t) {
#ifdef FCS_MASK_MINMAX   // measurement-only: the two-instruction clamp
    t = t < 0 ? 0 : (t > 32 ? 32 : t);
#else
    asm("v_med3_i32 %0, %1, 0, 32" : "=v"(t) : "v"(t));
#endif
    return w & (uint32_t)(0xFFFFFFFFull << t);
}

__device__ __forceinline__ uint32_t lds_rd(const uint8_t *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}

// Per-lane table bases for step4. Default: 32 replicas (replica = lane & 31), base0 = r*4 (T3 at
// +0, T2 at +128), base1 = 0x10000 | r*4 (T1, T0). FCS_LDS16 (measurement-only): one 256-B row per
// byte value e holding table slot b (the table of word byte b, T_{3-b}) x 16 replicas at
// e*256 + b*64 + (lane & 15)*4; lanes 16-31 of each half-wave rotate the chain word by 16 bits, so
// their lookup k uses slot k ^ 2 and the 32 lanes of one LDS pass hit 32 distinct banks.
__device__ __forceinline__ void table_bases(int lane, uint32_t &base0, uint32_t &base1) {
#ifdef FCS_LDS16
    const uint32_t r = (uint32_t)(lane & 15) * 4u, G = (lane & 16) ? 2u : 0u;
    base0 = r + G * 64u;
    base1 = r + (2u - G) * 64u;
#else
    const uint32_t r4 = (uint32_t)(lane & 31) * 4u;
    base0 = r4;
    base1 = 0x10000u | r4;
#endif
}

// One 4-byte step with the next word folded in: returns A_4(x) ^ wn, where
// A_4(x) = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3] -> 4 v_perm + 4 ds_read + 2 v_bitop3.
// base0 = r*4 (half 0: T3 at +0, T2 at +128), base1 = 0x10000 | r*4 (half 1: T1, T0).
__device__ __forceinline__ uint32_t step4(const uint8_t *lds, uint32_t x, uint32_t wn, uint32_t base0,
                                          uint32_t base1) {
#ifdef FCS_LDS16   // measurement-only build: 64 KiB table set (see table_bases)
    const uint32_t xr = __builtin_amdgcn_perm(x, x, (threadIdx.x & 16) ? 0x01000302u : 0x03020100u);
    const uint32_t a0 = __builtin_amdgcn_perm(xr, base0, 0x0C0C0400u);
    const uint32_t a1 = __builtin_amdgcn_perm(xr, base0, 0x0C0C0500u);
    const uint32_t a2 = __builtin_amdgcn_perm(xr, base1, 0x0C0C0600u);
    const uint32_t a3 = __builtin_amdgcn_perm(xr, base1, 0x0C0C0700u);
    const uint32_t t3 = lds_rd(lds, a0);
    const uint32_t t2 = lds_rd(lds, a1 + 64);
    const uint32_t t1 = lds_rd(lds, a2);
    const uint32_t t0 = lds_rd(lds, a3 + 64);
    return xor3(xor3(t3, t2, t1), t0, wn);
#else
    const uint32_t a0 = __builtin_amdgcn_perm(x, base0, 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(x, base0, 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(x, base1, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(x, base1, 0x0C020700u);
#if defined(FCS_ABL_NOLDS)   // measurement-only build: LDS reads replaced by cheap VALU
    return xor3(a0 ^ (a1 >> 3), (a2 << 5) ^ (a3 >> 1), wn);
#else
    const uint32_t t3 = lds_rd(lds, a0);
    const uint32_t t2 = lds_rd(lds, a1 + 128);
    const uint32_t t1 = lds_rd(lds, a2);
    const uint32_t t0 = lds_rd(lds, a3 + 128);
    return xor3(xor3(t3, t2, t1), t0, wn);
#endif
#endif
}

// XOR of 8 table values and one extra input: 4 v_bitop3.
__device__ __forceinline__ uint32_t xor9(const uint32_t (&r)[8], uint32_t extra) {
    return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), xor3(r[6], r[7], extra));
}

// A_{96 j}(s): this lane's own nibble tables (entry e of table t at kLdsLane + t*2048 + e*128 +
// (lane & 31)*4; the slot holds the table of lane & 15).
__device__ __forceinline__ uint32_t lane_shift(const uint8_t *lds, uint32_t s, uint32_t lanebase) {
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 7) ? (s >> (4 * t - 7)) : (s << (7 - 4 * t));
        r[t] = lds_rd(lds, ((sh & 0x780u) | lanebase) + t * 2048);
    }
    return xor9(r, 0u);
}

// A_n(s) for one n shared by all lanes (J = A_1536, H48 = A_48, H24 = A_24):
// entry e of nibble table t at REGION + t*64 + e*4; 16 entries span 16 banks -> conflict free.
// Returns A_n(s) ^ extra.
template <uint32_t REGION>
__device__ __forceinline__ uint32_t uniform_shift(const uint8_t *lds, uint32_t s, uint32_t extra) {
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        r[t] = lds_rd(lds, ((sh & 0x3Cu) | REGION) + t * 64);
    }
    return xor9(r, extra);
}

// XOR over each 16-lane row (one frame); every lane of the row ends with the row's XOR.
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    return v;
}

struct Item {
    uint64_t end;   // byte address one past the frame's last byte
    uint32_t len;
    uint32_t m;     // segments
};

template <bool VAR>
__device__ __forceinline__ Item frame_item(const KParams &p, uint64_t f) {
    Item it;
    if (VAR) {
        const uint32_t L = p.len[f];
        it.end = p.base + (p.off ? p.off[f] : f * p.stride) + L;
        it.len = L;
        it.m = L ? (L + (kSegBytes - 1)) / kSegBytes : 1u;
    } else {
        it.end = p.base + f * p.stride + p.flen;
        it.len = p.flen;
        it.m = p.fseg;
    }
    return it;
}

// Raw loads of one lane chunk (issued one item ahead of their use) and what is needed to
// interpret them. Loads are unconditional and stay inside [lo4, hi4): lanes with nothing to load
// read lo4; a window that starts before lo4 (front lane of a frame at the very start of the
// arena) is moved up to lo4 in a wave-uniform branch and shifted back after the data has landed
// (process()).
// CRC residue: ether_fcs(frame || LE32(ether_fcs(frame))) for every frame.
constexpr uint32_t kResidue = 0x2144DF1Cu;

// Result store for one frame per lane with st set; called by the whole wave (convergent).
// FCS mode: out[i] = FCS. Verify mode (ok != null; frames carry their FCS trailer): ok[i] = 1 iff
// the FCS over the whole frame equals the residue; non-matching frames are counted in the wave's
// LDS slot (lane 0 only touches it) and added to *bad once per wave at kernel exit (flush_bad), so
// an all-bad batch costs no atomics on the data path. Both outputs may be requested together.
// BAD: LDS byte offset of the per-wave counters (kLdsBad; the LDS-DMA kernel keeps them elsewhere).
template <uint32_t BAD = kLdsBad>
__device__ __forceinline__ uint64_t *wave_bad(const uint8_t *lds) {   // the kernels' own __shared__ array
    return reinterpret_cast<uint64_t *>(const_cast<uint8_t *>(lds) + BAD) + (threadIdx.x >> 6);
}

template <uint32_t BAD = kLdsBad>
__device__ __forceinline__ void emit(const KParams &p, const uint8_t *lds, bool st, uint64_t i, uint32_t fcs) {
    if (p.out != nullptr && st) p.out[i] = fcs;
    if (p.ok != nullptr) {
        const bool good = fcs == kResidue;
        if (st) p.ok[i] = good ? 1 : 0;
        const uint64_t m = __ballot(st && !good);
        if (m != 0 && (threadIdx.x & 63) == 0) *wave_bad<BAD>(lds) += (uint64_t)__popcll(m);
    }
}

template <uint32_t BAD = kLdsBad>
__device__ __forceinline__ void init_bad(const uint8_t *lds) {
    if ((threadIdx.x & 63) == 0) *wave_bad<BAD>(lds) = 0;
}

template <uint32_t BAD = kLdsBad>
__device__ __forceinline__ void flush_bad(const KParams &p, const uint8_t *lds) {
    if (p.ok != nullptr && (threadIdx.x & 63) == 0) {
        const uint64_t b = *wave_bad<BAD>(lds);
        if (b) atomicAdd(p.bad, (unsigned long long)b);
    }
}

// Chunk loads are issued at raised wave priority: a wave about to feed the memory pipe goes ahead
// of waves busy with CRC arithmetic (+1.6 % on 64 M x 1518, tools/ab.py). Scoped: the wave drops
// back to priority 0 right after its loads are issued.
#ifndef FCS_LOAD_PRIO
#define FCS_LOAD_PRIO 1
#endif
struct LoadPriority {
    __device__ __forceinline__ LoadPriority() { __builtin_amdgcn_s_setprio(FCS_LOAD_PRIO); }
    __device__ __forceinline__ ~LoadPriority() { __builtin_amdgcn_s_setprio(0); }
};

struct Chunk {
    u32x4a4 x[6];
    uint32_t x6;
    int zr;        // bytes from chunk start to frame start (segment 0); -1 inside; 96 = no data
    uint32_t r;    // chunk start & 3 (realignment)
    int dlead;     // dwords the load window was moved up to stay >= lo4 (0 = not moved)
};

template <bool VAR, bool TINY, bool SINGLE>
__device__ __forceinline__ void issue_chunk(const KParams &p, const Item &it, uint32_t k, int j,
                                            bool act, Chunk &c) {
    LoadPriority lp;
    int64_t cstart;
    if (SINGLE) {   // fixed length, one segment: zr does not depend on the frame
        cstart = (int64_t)it.end - (int64_t)kChunkBytes * (j + 1);
        const int z = kChunkBytes * (j + 1) - (int)p.flen;
        c.zr = z < -1 ? -1 : (z > kChunkBytes ? kChunkBytes : z);
    } else {
        cstart = (int64_t)it.end - (int64_t)kSegBytes * (int64_t)(it.m - 1 - k) -
                 (int64_t)kChunkBytes * (j + 1);
        const int64_t z = (k == 0) ? ((int64_t)(it.end - it.len) - cstart) : -1;
        c.zr = z < -1 ? -1 : (z > kChunkBytes ? kChunkBytes : (int)z);
    }
    c.r = (uint32_t)cstart & 3u;
    const bool need = act && c.zr < kChunkBytes;
    const uint64_t a = need ? ((uint64_t)cstart & ~3ull) : p.lo4;
    c.dlead = 0;
    if (TINY) {
        // Arena shorter than 192 B (host-selected variant): per-dword guarded loads.
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int q = 0; q <= kChunkWords; q++) {
            const uint64_t ad = a + 4 * q;
            d[q] = (need && ad >= p.lo4 && ad + 4 <= p.hi4) ? gload<uint32_t>(ad) : 0u;
        }
#pragma unroll
        for (int g = 0; g < 6; g++) c.x[g] = u32x4a4{d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]};
        c.x6 = d[kChunkWords];
        return;
    }
    // High side in bounds by construction: a + 96 <= chunk end <= hi4; the 25th dword (needed
    // only when r != 0) ends at ceil4(chunk end) <= hi4; when r == 0 dword 23 is re-read instead.
    // Low side: a window starting before lo4 (front lane of a frame at the arena start) is moved
    // up to lo4 as a whole; process() shifts the dwords back by dlead (wave-uniform, rare branch).
    uint64_t ab = a;
    if (__any(a < p.lo4)) {
        c.dlead = a < p.lo4 ? (int)((p.lo4 - a) >> 2) : 0;
        ab = a < p.lo4 ? p.lo4 : a;
    }
#ifdef FCS_ABL_COALESCED   // measurement-only build: same bytes per quarter, coalesced 256-B rows
    {
        // quarter's segment start, 16-B aligned, clamped to the arena: every read stays in
        // [lo16, sb + 1536) with sb + 1536 <= frame end (or lo16 + 1536 for idle/edge lanes).
        const uint64_t seg0 = (uint64_t)cstart + (uint64_t)kChunkBytes * (j + 1) - kSegBytes;
        const uint64_t lo16 = (p.lo4 + 15) & ~15ull;
        uint64_t sb = seg0 & ~15ull;
        sb = (need && sb >= lo16) ? sb : lo16;
        const uint64_t cb = sb + 16 * (uint64_t)j;
#pragma unroll
        for (int q = 0; q < 6; q++) c.x[q] = gload<u32x4a4>(cb + 256 * q);
        c.x6 = gload<uint32_t>(cb + 4);
        return;
    }
#endif
#pragma unroll
    for (int q = 0; q < 6; q++) c.x[q] = gload<u32x4a4>(ab + 16 * q);
    c.x6 = gload<uint32_t>(ab + ((c.r || c.dlead) ? 96 : 92));
}

// Undo the window move of issue_chunk: true dword q = loaded dword q - dlead (q >= dlead); dwords
// q < dlead lie before the arena start, hence before the frame start, and get masked anyway.
template <int N>
__device__ __forceinline__ void shift_up(uint32_t (&d)[N], int dlead) {
#pragma unroll
    for (int b = 16; b >= 1; b >>= 1) {
        const bool take = (dlead & b) != 0;
#pragma unroll
        for (int q = N - 1; q >= 0; q--) d[q] = take ? (q >= b ? d[q - b] : 0u) : d[q];
    }
}

// Hands out the units [0, U) of a launch to the waves of a persistent grid (wave-uniform state).
// Without a counter: wave wid of W takes wid, wid + W, ... (interleaved). With one (a zeroed device
// word, KParams::ctr): the first (100 - dyn_pct) % of the units that way, the rest in chunks of
// consecutive units from *ctr, sized by the work left (guided: left / 2W, clamped to cmin..cmax),
// each chunk requested when the previous one starts so the atomic's latency stays hidden.
#ifndef FCS_FIXED_CHUNK_MAX   // measurement-only overrides: largest dynamic chunk, in units
#define FCS_FIXED_CHUNK_MAX 64   // generic fixed kernel: units of 4 frames
#endif
#ifndef FCS_FIXED_DYN_PCT
#define FCS_FIXED_DYN_PCT 100    // generic fixed kernel: share of the units handed out dynamically
#endif
#ifndef FCS_FLAT_CHUNK_MAX
#define FCS_FLAT_CHUNK_MAX 16    // flat kernel: 64-frame windows
#endif
struct Dispenser {
    static constexpr uint64_t kEnd = ~0ull;
    unsigned long long *ctr;
    uint64_t U, W, wid, Is, Ks;
    uint64_t k = 0, ce = 0, pend = 0, psize = 0, seen = 0;
    uint32_t cmin, cmax;
    int lane;
    bool dyn = false;

    __device__ Dispenser(unsigned long long *ctr_, uint64_t U_, uint64_t W_, uint64_t wid_, int lane_,
                         uint32_t dyn_pct, uint32_t cmin_, uint32_t cmax_)
        : ctr(ctr_), U(U_), W(W_), wid(wid_), cmin(cmin_), cmax(cmax_), lane(lane_) {
        Is = ctr ? (U * (100 - dyn_pct) / 100) / W * W : U;   // statically assigned units in all
        Ks = wid < Is ? (Is - wid + W - 1) / W : 0;             // ... of this wave
    }
    __device__ void grab() {
        const uint64_t left = U - Is > seen ? U - Is - seen : 0;
        uint64_t sz = left / (2 * W);
        sz = sz < cmin ? cmin : (sz > cmax ? cmax : sz);
        uint64_t v = 0;
        if (lane == 0) v = atomicAdd(ctr, (unsigned long long)sz);
        pend = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
               (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
        psize = sz;
    }
    __device__ uint64_t take() {   // move to the requested chunk, request the one after it
        const uint64_t cb = Is + pend;
        seen = pend + psize;
        if (cb >= U) return kEnd;
        ce = cb + psize < U ? cb + psize : U;
        grab();
        return cb;
    }
    __device__ uint64_t first() {
        if (ctr) grab();   // the first dynamic chunk, requested while the static share runs
        if (Ks) return wid;
        if (!ctr) return kEnd;
        dyn = true;
        return take();
    }
    __device__ uint64_t next(uint64_t cur) {
        if (!dyn) {
            if (k + 1 < Ks) return wid + (++k) * W;
            if (!ctr) return kEnd;
            dyn = true;
            return take();
        }
        return cur + 1 < ce ? cur + 1 : take();
    }
};

template <bool VAR, bool TINY, bool SINGLE>
struct Lane {
    const KParams &p;
    const uint8_t *lds;
    int j;            // lane within the frame's 16
    uint32_t base0, base1, lanebase;
    uint64_t Q;       // frame slots in the grid
    Dispenser *D;     // fixed frames of any segment count: wave units of 4 frames (else null)
    uint32_t q;       // quarter of the wave (frame 4u + q of unit u)

    struct Pos {
        uint64_t f;
        uint64_t u;   // D's unit (D only)
        uint32_t k;
        bool act;
        Item it;
    };

    __device__ __forceinline__ Pos next(const Pos &c) const {
        Pos n = c;
        if (!VAR && !SINGLE && D != nullptr) {
            // every frame has p.fseg segments: the quarters wrap together, the unit step is uniform
            n.k = c.k + 1;
            if (n.k >= p.fseg) {
                n.k = 0;
                n.u = c.u == Dispenser::kEnd ? c.u : D->next(c.u);
                n.f = n.u == Dispenser::kEnd ? p.n : 4 * n.u + q;
            }
        } else if (SINGLE) {
            n.f = c.f + Q;
            n.k = 0;
        } else {
            n.k = c.k + 1;
            if (n.k >= c.it.m) {
                n.f = c.f + Q;
                n.k = 0;
            }
        }
        n.act = c.act && n.f < p.n;
        if (SINGLE || (n.act && n.k == 0)) n.it = frame_item<VAR>(p, n.f);
        return n;
    }

    // Consume one chunk: realign, mask, run the two chains, finish the frame if last.
    __device__ __forceinline__ void process(const Pos &c, const Chunk &ch, uint32_t &s) const {
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int q = 0; q < 6; q++) {
            d[4 * q] = ch.x[q].x;
            d[4 * q + 1] = ch.x[q].y;
            d[4 * q + 2] = ch.x[q].z;
            d[4 * q + 3] = ch.x[q].w;
        }
        d[kChunkWords] = ch.x6;
        if (!TINY && __any(ch.dlead)) shift_up(d, ch.dlead);   // arena start only; uniform
        uint32_t w[kChunkWords];
#pragma unroll
        for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], ch.r);
#ifdef FCS_ABL_NOCOMPUTE   // measurement-only build: loads + realign
        {
            uint32_t acc = 0;
#pragma unroll
            for (int i = 0; i < kChunkWords; i++) acc ^= w[i];
            s ^= acc;
            if (c.act && j == 15 && s == 0x12345678u) p.out[c.f] = s;
            return;
        }
#endif
        uint32_t x0 = 0;
        const bool first = SINGLE || c.k == 0;
        if (first) {
#pragma unroll
            for (int i = 0; i < kChunkWords; i++) {
                // uniform bound: words no front lane can mask are skipped. SINGLE launches only when
                // zmax <= 32 (host), so at most 8 loop-invariant masks stay live in registers.
                if ((!SINGLE || i < kSingleMaskWords) && 4 * i < (int)p.zmax) {
                    int t = ch.zr - 4 * i;
                    t = t < 0 ? 0 : (t > 4 ? 4 : t);
                    w[i] &= (uint32_t)(0xFFFFFFFFull << (8 * t));
                }
            }
            const int zi = ch.zr < 0 ? 0 : (ch.zr > kChunkBytes - 1 ? kChunkBytes - 1 : ch.zr);
            const uint32_t iv = lds_rd(lds, kLdsInv + 4u * (uint32_t)zi);
            x0 = (ch.zr >= 0 && ch.zr < kChunkBytes) ? iv : 0u;
        }
#if FCS_CHAINS == 2
        // Two independent 12-word chains, merged with A_48.
        uint32_t xa = x0 ^ w[0], xb = w[12];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            xa = step4(lds, xa, i < 11 ? w[i + 1] : 0u, base0, base1);
            xb = step4(lds, xb, i < 11 ? w[13 + i] : 0u, base0, base1);
        }
        const uint32_t r = uniform_shift<kLdsH48>(lds, xa, xb);
#else
        // Four independent 6-word chains (ILP 4 on the LDS/VALU latency), merged as a tree.
        uint32_t xa = x0 ^ w[0], xb = w[6], xc = w[12], xd = w[18];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            xa = step4(lds, xa, i < 5 ? w[i + 1] : 0u, base0, base1);
            xb = step4(lds, xb, i < 5 ? w[7 + i] : 0u, base0, base1);
            xc = step4(lds, xc, i < 5 ? w[13 + i] : 0u, base0, base1);
            xd = step4(lds, xd, i < 5 ? w[19 + i] : 0u, base0, base1);
        }
        const uint32_t ab = uniform_shift<kLdsH24>(lds, xa, xb);
        const uint32_t cd = uniform_shift<kLdsH24>(lds, xc, xd);
        const uint32_t r = uniform_shift<kLdsH48>(lds, ab, cd);
#endif
        s = first ? r : uniform_shift<kLdsJump>(lds, s, r);

        const bool last = c.act && (SINGLE || c.k + 1 == c.it.m);
#ifdef FCS_ABL_NOFINAL   // measurement-only build: no lane shift / reduction
        if (last && j == 15) p.out[c.f] = s;
        return;
#endif
        if (__any(last)) {
            uint32_t v = last ? lane_shift(lds, s, lanebase) : 0u;
            v = row_xor(v);
            emit(p, lds, last && j == 15, c.f, c.it.len ? ~v : 0u);
        }
    }
};

// Stage the constant tables into LDS (once per workgroup; grids are persistent).
template <int NT>
__device__ __forceinline__ void stage_tables(const KParams &p, uint8_t *lds) {
    const int tid = threadIdx.x;
    // data: 8192 x 16 B; each b128 store = 4 replicas of one entry
#ifdef FCS_LDS16
    for (int i = tid; i < 4096; i += NT) {   // row e = i >> 4; 16-B store q = i & 15 -> slot q >> 2
        const uint32_t v = p.blob[kBlobSlice + 256 * (3 - ((i & 15) >> 2)) + (i >> 4)];
        u32x4 vv = {v, v, v, v};
        *reinterpret_cast<u32x4 *>(lds + kLdsData + (uint32_t)i * 16) = vv;
    }
#else
    for (int i = tid; i < 8192; i += NT) {
        const int h = i >> 12;            // 64 KiB half
        const int b = (i >> 4) & 255;     // entry
        const int odd = (i >> 3) & 1;     // +128 slot
        // half 0: T3 (+0), T2 (+128); half 1: T1 (+0), T0 (+128)
        const int k = h == 0 ? (odd ? 2 : 3) : (odd ? 0 : 1);
        const uint32_t v = p.blob[kBlobSlice + 256 * k + b];
        u32x4 vv = {v, v, v, v};
        *reinterpret_cast<u32x4 *>(lds + kLdsData + (uint32_t)i * 16) = vv;
    }
#endif
    const uint32_t *src = p.blob + kBlobLane;
    uint32_t *dst = reinterpret_cast<uint32_t *>(lds + kLdsLane);
    for (int i = tid; i < (int)(kBlobFlat - kBlobLane); i += NT) dst[i] = src[i];
    __syncthreads();
}

// Flat variable-length kernel staging: the same data and uniform tables, and the chunk-shift
// tables C_c in place of the per-lane tables.
__device__ __forceinline__ void stage_tables_flat(const KParams &p, uint8_t *lds) {
    const int tid = threadIdx.x;
#ifdef FCS_LDS16
    for (int i = tid; i < 4096; i += kWgThreads) {
        const uint32_t v = p.blob[kBlobSlice + 256 * (3 - ((i & 15) >> 2)) + (i >> 4)];
        u32x4 vv = {v, v, v, v};
        *reinterpret_cast<u32x4 *>(lds + kLdsData + (uint32_t)i * 16) = vv;
    }
#else
    for (int i = tid; i < 8192; i += kWgThreads) {
        const int h = i >> 12, b = (i >> 4) & 255, odd = (i >> 3) & 1;
        const int k = h == 0 ? (odd ? 2 : 3) : (odd ? 0 : 1);
        const uint32_t v = p.blob[kBlobSlice + 256 * k + b];
        u32x4 vv = {v, v, v, v};
        *reinterpret_cast<u32x4 *>(lds + kLdsData + (uint32_t)i * 16) = vv;
    }
#endif
    uint32_t *dst = reinterpret_cast<uint32_t *>(lds + kLdsJump);
    for (int i = tid; i < (int)(kBlobFlat - kBlobJump); i += kWgThreads) dst[i] = p.blob[kBlobJump + i];
    uint32_t *fl = reinterpret_cast<uint32_t *>(lds + kLdsFlat);
    for (int i = tid; i < (int)(kFlatBytes / 4); i += kWgThreads) fl[i] = p.blob[kBlobFlat + i];
    __syncthreads();
}

// The quarter-wave-per-frame loop of one workgroup (`blk` of `nblk`), tables already in LDS.
template <bool VAR, bool TINY, bool SINGLE, int NT>
__device__ __forceinline__ void fcs_body(const KParams &p, const uint8_t *lds, uint32_t blk, uint32_t nblk) {
    const int lane = threadIdx.x & 63;
    const int j = lane & (kGroup - 1);
    const uint32_t r4 = (uint32_t)(lane & 31) * 4u;
    uint32_t tb0, tb1;
    table_bases(lane, tb0, tb1);
    // Fixed frames: a wave's unit is 4 consecutive frames (one per quarter), units from the
    // dispenser (interleaved over the grid's waves, the tail dynamic when the host gave a counter).
    constexpr bool kUnits = !VAR && !SINGLE && !TINY;
    Dispenser D(kUnits ? p.ctr : nullptr, (p.n + 3) >> 2, (uint64_t)nblk * (NT / 64),
                (uint64_t)blk * (NT / 64) + (threadIdx.x >> 6), lane, FCS_FIXED_DYN_PCT, 1, FCS_FIXED_CHUNK_MAX);
    Lane<VAR, TINY, SINGLE> L{p, lds, j, tb0, tb1, kLdsLane | r4, (uint64_t)nblk * kSlotsPerWg<NT>,
                              kUnits ? &D : nullptr, (uint32_t)(threadIdx.x >> 4) & 3u};

    typename Lane<VAR, TINY, SINGLE>::Pos A, B;
    if (kUnits) {
        A.u = D.first();
        A.f = A.u == Dispenser::kEnd ? p.n : 4 * A.u + L.q;
    } else {
        A.u = 0;
        A.f = ((uint64_t)blk * kSlotsPerWg<NT>) + (threadIdx.x / kGroup);
    }
    A.k = 0;
    A.act = A.f < p.n;
    A.it = (SINGLE || A.act) ? frame_item<VAR>(p, A.f) : Item{0, 0, 1};
    Chunk CA, CB;
    issue_chunk<VAR, TINY, SINGLE>(p, A.it, A.k, j, A.act, CA);
    uint32_t s = 0;

#ifndef FCS_PREFETCH_DEPTH
#define FCS_PREFETCH_DEPTH 2
#endif
#if FCS_PREFETCH_DEPTH == 2
    // Two items in flight per lane: process one while the other's loads are outstanding.
    while (__any(A.act)) {
        B = L.next(A);
        issue_chunk<VAR, TINY, SINGLE>(p, B.it, B.k, j, B.act, CB);
        L.process(A, CA, s);
        if (!__any(B.act)) break;
        A = L.next(B);
        issue_chunk<VAR, TINY, SINGLE>(p, A.it, A.k, j, A.act, CA);
        L.process(B, CB, s);
    }
#else
    // Three chunk buffers: while one item is processed the next two have their loads in flight.
    typename Lane<VAR, TINY, SINGLE>::Pos C;
    Chunk CC;
    B = L.next(A);
    issue_chunk<VAR, TINY, SINGLE>(p, B.it, B.k, j, B.act, CB);
    for (;;) {
        if (!__any(A.act)) break;
        C = L.next(B);
        issue_chunk<VAR, TINY, SINGLE>(p, C.it, C.k, j, C.act, CC);
        L.process(A, CA, s);
        if (!__any(B.act)) break;
        A = L.next(C);
        issue_chunk<VAR, TINY, SINGLE>(p, A.it, A.k, j, A.act, CA);
        L.process(B, CB, s);
        if (!__any(C.act)) break;
        B = L.next(A);
        issue_chunk<VAR, TINY, SINGLE>(p, B.it, B.k, j, B.act, CB);
        L.process(C, CC, s);
    }
#endif
}

template <bool VAR, bool TINY, bool SINGLE, int NT>
__global__ __launch_bounds__(NT, 1) void fcs_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    stage_tables<NT>(p, lds);
    init_bad(lds);
    fcs_body<VAR, TINY, SINGLE, NT>(p, lds, blockIdx.x, gridDim.x);
    flush_bad(p, lds);
}


// ---------------------------------------------------------------------------------------------
// Fixed length, one segment, at most 32 leading garbage bytes in the front lane (host-selected:
// 1504 <= len <= 1536, which covers the 1518-B benchmark frames). The generic kernel's work per
// item, strength-reduced: the frame end advances by a constant, the per-lane chunk offset, front
// masks and INV start value are loop invariants, and only a wave's first item can touch the
// arena start, so the edge repair is peeled out of the loop.
// ---------------------------------------------------------------------------------------------
struct Raw {
    u32x4a4 x[6];
    uint32_t x6;
};

__device__ __forceinline__ uint64_t stamp() {
    return __builtin_amdgcn_s_memtime();
}

struct SingleLane {
    uint64_t *dbg;
    const KParams *kp;
    const uint8_t *lds;
    int j;
    uint32_t base0, base1, lanebase, x0, zmax;
    uint32_t m[kSingleMaskWords];

    template <bool EDGE>
    __device__ __forceinline__ void process(const Raw &c, uint32_t r, int dlead, bool act, uint64_t fi) const {
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int q = 0; q < 6; q++) {
            d[4 * q] = c.x[q].x;
            d[4 * q + 1] = c.x[q].y;
            d[4 * q + 2] = c.x[q].z;
            d[4 * q + 3] = c.x[q].w;
        }
        d[kChunkWords] = c.x6;
        if (EDGE && __any(dlead)) shift_up(d, dlead);
#ifdef FCS_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts0 = stamp();
        __builtin_amdgcn_sched_barrier(0);
#endif
        uint32_t w[kChunkWords];
#pragma unroll
#ifdef FCS_ABL_NOALIGN   // measurement-only build: no realignment (wrong CRCs unless r == 0)
        for (int i = 0; i < kChunkWords; i++) w[i] = d[i];
#else
        for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], r);
#endif
#pragma unroll
        for (int i = 0; i < kSingleMaskWords; i++)
            if (4 * i < (int)zmax) w[i] &= m[i];
#ifdef FCS_SINGLE_ONE_CHAIN   // one 24-word chain: no A_48 merge (8 fewer LDS reads per item)
        uint32_t xa = x0 ^ w[0];
#pragma unroll
        for (int i = 0; i < 24; i++) xa = step4(lds, xa, i < 23 ? w[i + 1] : 0u, base0, base1);
        uint32_t v = lane_shift(lds, xa, lanebase);
#else
        uint32_t xa = x0 ^ w[0], xb = w[12];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            xa = step4(lds, xa, i < 11 ? w[i + 1] : 0u, base0, base1);
            xb = step4(lds, xb, i < 11 ? w[13 + i] : 0u, base0, base1);
        }
#ifdef FCS_STAMPS
        asm volatile("" ::"v"(xa), "v"(xb));
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts1 = stamp();
        __builtin_amdgcn_sched_barrier(0);
#endif
        uint32_t v = lane_shift(lds, uniform_shift<kLdsH48>(lds, xa, xb), lanebase);
#endif
        v = row_xor(v);
        emit(*kp, lds, act && j == 15, fi, ~v);
#ifdef FCS_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts2 = stamp();
        if (dbg != nullptr && (threadIdx.x & 63) == 0) {
            const uint32_t wv = blockIdx.x * (kFixedWgThreads / 64) + (threadIdx.x >> 6);
            atomicAdd((unsigned long long *)&dbg[wv * 4 + 0], (unsigned long long)(ts1 - ts0));
            atomicAdd((unsigned long long *)&dbg[wv * 4 + 1], (unsigned long long)(ts2 - ts0));
            atomicAdd((unsigned long long *)&dbg[wv * 4 + 2], 1ull);
            atomicAdd((unsigned long long *)&dbg[wv * 4 + 3], (unsigned long long)ts2);
        }
#endif
    }
};

__device__ __forceinline__ void issue_raw(uint64_t a, uint32_t r, Raw &c) {
    LoadPriority lp;
#pragma unroll
    for (int q = 0; q < 6; q++) c.x[q] = gload<u32x4a4>(a + 16 * q);
    c.x6 = gload<uint32_t>(a + (r ? 96 : 92));   // 25th dword only matters when r != 0
}

__global__ __launch_bounds__(kFixedWgThreads, 1) void fcs_single_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    stage_tables<kFixedWgThreads>(p, lds);
    init_bad(lds);

    const int lane = threadIdx.x & 63;
    const int j = lane & (kGroup - 1);
    const uint32_t r4 = (uint32_t)(lane & 31) * 4u;
    SingleLane S;
    S.dbg = p.dbg;
    S.kp = &p;
    S.lds = lds;
    S.j = j;
    table_bases(lane, S.base0, S.base1);
    S.lanebase = kLdsLane | r4;
    S.zmax = p.zmax;
    const uint32_t loff = (uint32_t)kChunkBytes * (uint32_t)(j + 1);   // chunk start = end - loff
    {
        int zr = (int)loff - (int)p.flen;
        zr = zr < -1 ? -1 : (zr > kChunkBytes ? kChunkBytes : zr);
#pragma unroll
        for (int i = 0; i < kSingleMaskWords; i++) {
            int t = zr - 4 * i;
            t = t < 0 ? 0 : (t > 4 ? 4 : t);
            S.m[i] = (uint32_t)(0xFFFFFFFFull << (8 * t));
        }
        const uint32_t iv = lds_rd(lds, kLdsInv + 4u * (uint32_t)(zr < 0 ? 0 : (zr > kChunkBytes - 1 ? kChunkBytes - 1 : zr)));
        S.x0 = (zr >= 0 && zr < kChunkBytes) ? iv : 0u;
    }

#ifdef FCS_BLOCKED   // measurement-only build: each workgroup walks its own contiguous frame range
    const uint64_t Q = (uint64_t)kSlotsPerWg<kFixedWgThreads>;
    const uint64_t per = ((p.n + Q - 1) / Q + gridDim.x - 1) / gridDim.x;   // items per workgroup
    const uint64_t f0 = (uint64_t)blockIdx.x * per * Q + threadIdx.x / kGroup;
    const uint64_t lim = (uint64_t)(blockIdx.x + 1) * per * Q < p.n ? (uint64_t)(blockIdx.x + 1) * per * Q : p.n;
    int rem = f0 < lim ? (int)((lim - 1 - f0) / Q) + 1 : 0;
#else
#ifdef FCS_XCD   // measurement-only build: neighbouring frame slots on one XCD (round-robin dispatch)
    const uint32_t wg = (gridDim.x & 7) ? blockIdx.x : (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
#else
    const uint32_t wg = blockIdx.x;
#endif
    const uint64_t Q = (uint64_t)gridDim.x * kSlotsPerWg<kFixedWgThreads>;
    const uint64_t f0 = (uint64_t)wg * kSlotsPerWg<kFixedWgThreads> + threadIdx.x / kGroup;
    int rem = f0 < p.n ? (int)((p.n - 1 - f0) / Q) + 1 : 0;   // items left for this frame slot
#endif
    uint64_t end = p.base + f0 * p.stride + p.flen;
    const uint64_t dend = Q * p.stride;
    uint64_t fi = f0;   // frame index of the item being processed

    // ---- first item: the only one that can start before the arena (frame 0's front lane) ----
    Raw A, B;
    int dlead = 0;
    uint32_t rA = (uint32_t)end & 3u;
    {
        const uint64_t a = rem > 0 ? ((end - loff) & ~3ull) : p.lo4;
        uint64_t ab = a;
        if (__any(a < p.lo4)) {
            dlead = a < p.lo4 ? (int)((p.lo4 - a) >> 2) : 0;
            ab = a < p.lo4 ? p.lo4 : a;
        }
        LoadPriority lp;
#pragma unroll
        for (int q = 0; q < 6; q++) A.x[q] = gload<u32x4a4>(ab + 16 * q);
        A.x6 = gload<uint32_t>(ab + ((rA || dlead) ? 96 : 92));
    }
    uint64_t endB = end + dend;
    uint32_t rB = (uint32_t)endB & 3u;
    issue_raw(rem > 1 ? ((endB - loff) & ~3ull) : p.lo4, rB, B);
    S.process<true>(A, rA, dlead, rem > 0, fi);
    rem -= 1;
    end = endB;
    fi += Q;

    // ---- steady state: two items in flight per lane ----
    while (__any(rem > 0)) {
        const uint64_t endA = end + dend;
        rA = (uint32_t)endA & 3u;
        issue_raw(rem > 1 ? ((endA - loff) & ~3ull) : p.lo4, rA, A);
        S.process<false>(B, rB, 0, rem > 0, fi);
        rem -= 1;
        end = endA;
        fi += Q;
        if (!__any(rem > 0)) break;
        endB = end + dend;
        rB = (uint32_t)endB & 3u;
        issue_raw(rem > 1 ? ((endB - loff) & ~3ull) : p.lo4, rB, B);
        S.process<false>(A, rA, 0, rem > 0, fi);
        rem -= 1;
        end = endB;
        fi += Q;
    }
    flush_bad(p, lds);
}


// ---------------------------------------------------------------------------------------------
// Fixed length, one segment, frames staged through LDS by DMA (fcs_dma_kernel; host-selected for
// kDmaMinLen..kDmaCover bytes, e.g. the 1518-B benchmark frames, when four consecutive frames fit
// a 6 KiB slot: fixed_dma()).
// A wave's item is four consecutive frames, as in fcs_single_kernel. The wave copies the item's
// bytes into one of its LDS slots with six global_load_lds_dwordx4 (each 1 KiB contiguous:
// coalesced rows, no VGPR destination, non-temporal since every line is read exactly once), then
// lane c of each frame reads its 96-byte window [E - e_c - 96, E - e_c) from the slot (25 dwords,
// realigned with v_alignbyte; the window offsets e_c = dma_end_off(c) put one frame's 16 windows on
// 16 distinct banks) and runs two slice-by-4 chains, the A_48 merge, the lane shift A_{e_c} and the
// row XOR. One slot per wave, 16 waves per CU: the DMA of a wave's next item is issued as soon as
// the current item's words are in registers, so it lands while the CRC work runs.
// Items: a static interleaved share (item wid + k W for wave wid of W) and, for large batches
// (p.ctr != null), a dynamic tail: the remaining items are handed out in chunks by a device
// counter, chunk sizes shrinking with the work left (guided), the next chunk requested one chunk
// ahead. Without it the waves' finishing times spread over 18 % of the kernel (slower XCDs and
// CUs), and the kernel ends with the slowest (tools/stamps_dma.py).
//
// LDS (160 KiB): a 64 KiB table image of 256 rows of 256 B (row = byte value e) and the slots.
//   row bytes [0, 128): slice tables, slot s = T_{3-s}[e] x 8 replicas (lookups: step4_l8);
//   row bytes [128, 256) ("hole" e): hole 16 t + n = nibble n of the lane tables' table t for the
//     32 lane slots; holes 128.. the chain-merge tables, then INV, then the verify counters.
// ---------------------------------------------------------------------------------------------
#ifndef FCS_DMA_CHAINS   // independent chains per lane window (2, 3, 4 or 6; measurement override)
#define FCS_DMA_CHAINS 2
#endif
constexpr int kDmaChains = FCS_DMA_CHAINS;
constexpr int kDmaChainWords = kChunkWords / kDmaChains;
static_assert(kChunkWords % kDmaChains == 0 && kDmaChainWords % 2 == 0, "chains of an even word count");
constexpr uint32_t kDmaHole = 128;                                  // byte offset of a row's hole
__host__ __device__ constexpr uint32_t dma_hole(uint32_t q) { return q * 256u + kDmaHole; }
constexpr uint32_t kDmaMergeHole = 128;                             // 4 holes per merge table
constexpr uint32_t kDmaInvHole = kDmaMergeHole + 4 * 5;             // 3 holes: INV[0..95]
constexpr uint32_t kDmaBad = dma_hole(kDmaInvHole + 3);            // 16 x 8 B
constexpr uint32_t kDmaRing = 65536;                                // slots start after the tables
constexpr int kDmaWaves = kDmaWgThreads / 64;
constexpr uint32_t kDmaLdsBytes = kDmaRing + (uint32_t)kDmaWaves * (kDmaPair ? 2u : 1u) * kDmaItemBytes;
static_assert(kDmaLdsBytes <= 163840, "LDS per CU");
static_assert(kDmaChains - 1 <= 5, "merge holes");
#ifndef FCS_DMA_AUX   // cache policy of the slot DMA (2 = nt; measurement-only override)
#define FCS_DMA_AUX 2
#endif
#ifndef FCS_DMA_DYN_PCT   // share of the items handed out dynamically when p.ctr is set
#define FCS_DMA_DYN_PCT 100
#endif
#ifndef FCS_DMA_CHUNK_MAX   // largest dynamic chunk (items); measurement-only override
#define FCS_DMA_CHUNK_MAX 64
#endif

// One slice-by-4 step against the 32 KiB slice tables: T_{3-s}[e] at e * 256 + s * 32 + replica * 4
// (replica = lane & 7). ds_read_b32 banks are the dword address mod 32, so the 4 slots x 8
// replicas of a row are the 32 banks. Lane group h = (lane >> 3) & 3 looks byte k ^ h up in slot
// k ^ h at its k-th lookup, so the four 8-lane groups of a 32-lane access use four different
// slots and every lookup hits 32 distinct banks. Byte and slot are per-lane constants of the
// v_perm that forms the address: selector SEL[k] picks byte k ^ h of x, base B[k] = replica * 4 +
// 32 * (k ^ h).
__device__ __forceinline__ uint32_t step4_l8(const uint8_t *lds, uint32_t x, uint32_t wn, const uint32_t (&B)[4],
                                             const uint32_t (&SEL)[4]) {
#ifdef FCS_DMA_ABL_NOLDS   // measurement-only: lookups replaced by VALU on the addresses (wrong FCS)
    const uint32_t a0 = __builtin_amdgcn_perm(x, B[0], SEL[0]), a1 = __builtin_amdgcn_perm(x, B[1], SEL[1]);
    const uint32_t a2 = __builtin_amdgcn_perm(x, B[2], SEL[2]), a3 = __builtin_amdgcn_perm(x, B[3], SEL[3]);
    return xor3(xor3(a0, a1 << 3, a2 >> 1), a3 << 7, wn);
#else
    const uint32_t t3 = lds_rd(lds, __builtin_amdgcn_perm(x, B[0], SEL[0]));
    const uint32_t t2 = lds_rd(lds, __builtin_amdgcn_perm(x, B[1], SEL[1]));
    const uint32_t t1 = lds_rd(lds, __builtin_amdgcn_perm(x, B[2], SEL[2]));
    const uint32_t t0 = lds_rd(lds, __builtin_amdgcn_perm(x, B[3], SEL[3]));
    return xor3(xor3(t3, t2, t1), t0, wn);
#endif
}

// A_{e_c}(s) from the lane tables in the holes: nibble n of table t at hole 16 t + n, slot lane & 31.
__device__ __forceinline__ uint32_t lane_shift_dma(const uint8_t *lds, uint32_t s, uint32_t lanebase) {
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 8) ? (s >> (4 * t - 8)) : (s << (8 - 4 * t));
        r[t] = lds_rd(lds, ((sh & 0xF00u) | lanebase) + (uint32_t)t * 4096u);
    }
    return xor9(r, 0u);
}

// Merge table m (A_{4 CL (m + 1)}): nibble table t at hole kDmaMergeHole + 4 m + t / 2, +64 (t odd).
__device__ __forceinline__ uint32_t merge_shift_dma(const uint8_t *lds, int m, uint32_t s, uint32_t extra) {
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        const uint32_t base = dma_hole(kDmaMergeHole + 4u * (uint32_t)m + (uint32_t)(t >> 1)) + 64u * (uint32_t)(t & 1);
        r[t] = lds_rd(lds, (sh & 0x3Cu) | base);
    }
    return xor9(r, extra);
}

// The slot DMA: six 1 KiB rows from two address registers. The instruction's offset (13-bit,
// 0 .. 3 KiB here) applies to the global AND the LDS address, so each group of rows passes the
// same LDS base (one M0 value).
// The first and last row of an item share their 128-B lines with the neighbouring items: those
// two rows keep the default cache policy (the line stays in L2 for the neighbour), the middle
// rows are non-temporal; the last row is trimmed to the lanes the item's bytes reach. Both +1.1 %
// on 64 M x 1518 B (tools/ab.py).
#ifndef FCS_DMA_EDGE_AUX   // measurement-only override
#define FCS_DMA_EDGE_AUX 0
#endif
// TRIM_ALL (segmented kernel, whose items can be shorter than 5 KiB): every row only as far as
// the item's bytes reach.
template <bool TRIM_ALL = false>
__device__ __forceinline__ void dma_item(const uint8_t *slot, uint64_t src, int lane, uint32_t need) {
    typedef __attribute__((address_space(3))) void lds_void;
    static_assert(kDmaItemBytes == 6 * 1024, "six rows");
    const uint64_t a = src + 16 * (uint64_t)lane, b = a + 4096;
    lds_void *la = (lds_void *)slot, *lb = (lds_void *)(slot + 4096);
    const uint32_t o = 16u * (uint32_t)lane;
    if (!TRIM_ALL || o < need)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 0, FCS_DMA_EDGE_AUX);
    if (!TRIM_ALL || 1024u + o < need)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 1024, FCS_DMA_AUX);
    if (!TRIM_ALL || 2048u + o < need)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 2048, FCS_DMA_AUX);
    if (!TRIM_ALL || 3072u + o < need)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 3072, FCS_DMA_AUX);
    if (!TRIM_ALL || 4096u + o < need)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(b), lb, 16, 0, FCS_DMA_AUX);
#ifndef FCS_DMA_NO_TRIM   // measurement-only: FCS_DMA_NO_TRIM loads the whole last row
    if (5120u + o < need)
#endif
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(b), lb, 16, 1024, FCS_DMA_EDGE_AUX);
    (void)need;
}

// Table image of the LDS-DMA kernels: slice tables (16-B stores of one value: 4 replicas), lane
// tables, merge tables, INV.
template <int NT = kDmaWgThreads>
__device__ __forceinline__ void stage_dma_tables(const KParams &p, uint8_t *lds, int tid) {
    for (int i = tid; i < 2048; i += NT) {   // row e = i >> 3; store j = i & 7 -> slot j >> 1
        const uint32_t v = p.blob[kBlobSlice + 256 * (3 - ((i & 7) >> 1)) + (i >> 3)];
        u32x4 vv = {v, v, v, v};
        *reinterpret_cast<u32x4 *>(lds + (uint32_t)(i >> 3) * 256u + (uint32_t)(i & 7) * 16u) = vv;
    }
    for (int i = tid; i < 4096; i += NT)   // [t][n][slot]: hole 16 t + n
        *reinterpret_cast<uint32_t *>(lds + dma_hole((uint32_t)i >> 5) + (uint32_t)(i & 31) * 4u) = p.blob[kBlobLaneDma + i];
    for (int i = tid; i < 128 * (kDmaChains - 1); i += NT) {   // merge table m = A_{4 CL (m + 1)}
        const int m = i >> 7, t = (i >> 4) & 7, e = i & 15;
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kDmaMergeHole + 4u * (uint32_t)m + (uint32_t)(t >> 1)) +
                                      64u * (uint32_t)(t & 1) + 4u * (uint32_t)e) =
            p.blob[kBlobMerge + ((m + 1) * (kDmaChainWords / 2) - 1) * 128 + (i & 127)];
    }
    for (int i = tid; i < kChunkBytes; i += NT)
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kDmaInvHole + (uint32_t)i / 32u) + (uint32_t)(i % 32) * 4u) =
            p.blob[kBlobInv + i];
}

// MW: words a front mask can touch (host-selected: 2 when the front lane masks at most 8 bytes,
// i.e. len >= 1516, else kSingleMaskWords).
// STREAM: the measurement form behind fcs_dma_stream_dev: the same slot DMA, schedule and window
// reads, no CRC work (bench.py's LDS-DMA read ceiling beside the plain read stream).
template <int MW, bool STREAM>
__global__ __launch_bounds__(kDmaWgThreads, 1) void fcs_dma_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDmaLdsBytes];
    const int tid = threadIdx.x;
    stage_dma_tables(p, lds, tid);
    init_bad<kDmaBad>(lds);
    __syncthreads();

    const int lane = tid & 63;
    const int c = lane & (kGroup - 1);     // chunk index back from the frame end
    const int g = lane >> 4;               // frame of the item
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint8_t *slot0 = lds + kDmaRing + (uint32_t)wave * (kDmaPair ? 2u : 1u) * kDmaItemBytes;
    const uint32_t h = (uint32_t)(lane >> 3) & 3u, r4 = (uint32_t)(lane & 7) * 4u;
    const uint32_t B[4] = {r4 + 32u * (0u ^ h), r4 + 32u * (1u ^ h), r4 + 32u * (2u ^ h), r4 + 32u * (3u ^ h)};
    const uint32_t SEL[4] = {0x0C0C0400u + ((0u ^ h) << 8), 0x0C0C0400u + ((1u ^ h) << 8),
                             0x0C0C0400u + ((2u ^ h) << 8), 0x0C0C0400u + ((3u ^ h) << 8)};
    const uint32_t lanebase = kDmaHole + (uint32_t)(lane & 31) * 4u;

    // loop invariants: window offset within the item, front masks, INV start of the front lane
    const uint32_t ec = dma_end_off(c);
    const int64_t klane = (int64_t)g * (int64_t)p.stride + (int64_t)p.flen - (int64_t)ec - kChunkBytes;
    const int zc = (c == kGroup - 1) ? (int)(kDmaCover - p.flen) : (dma_short_lane(c) ? 4 : 0);
    static_assert(MW >= 1 && MW <= kSingleMaskWords, "mask words");
    uint32_t m[MW];
#pragma unroll
    for (int i = 0; i < MW; i++) {
        int t = zc - 4 * i;
        t = t < 0 ? 0 : (t > 4 ? 4 : t);
        m[i] = (uint32_t)(0xFFFFFFFFull << (8 * t));
    }
    const uint32_t x0 = (c == kGroup - 1) ? lds_rd(lds, dma_hole(kDmaInvHole + (uint32_t)zc / 32u) + (uint32_t)(zc % 32) * 4u)
                                          : 0u;

    const uint64_t lo16 = p.lo4 & ~15ull;
    const uint64_t smax = ((p.hi4 + 15) & ~15ull) - kDmaItemBytes;   // last slot start inside the arena
    auto slot_src = [&](uint64_t S) {
        const uint64_t a = S & ~15ull;
        return a < lo16 ? lo16 : (a > smax ? smax : a);
    };
    // ---- items (4 frames each), from the dispenser ----
    constexpr uint64_t kEnd = Dispenser::kEnd;
    Dispenser D(p.ctr, (p.n + 3) >> 2, (uint64_t)gridDim.x * kDmaWaves,
                (uint64_t)blockIdx.x * kDmaWaves + (uint64_t)wave, lane, FCS_DMA_DYN_PCT, 4, FCS_DMA_CHUNK_MAX);
    auto item_start = [&](uint64_t i) { return p.base + 4 * i * p.stride; };   // first frame of item i
    // slot bytes an item's windows read: up to its last frame's end plus the realignment dword
    auto item_need = [&](uint64_t S, uint64_t src) {
        const uint64_t e = S + 3 * p.stride + p.flen + 4 - src;
        return (uint32_t)(e < (uint64_t)kDmaItemBytes ? e : (uint64_t)kDmaItemBytes);
    };
    auto dma_of = [&](const uint8_t *slot, uint64_t i) {
#ifdef FCS_DMA_PRIO   // measurement-only: the slot DMA issued at raised wave priority
        LoadPriority lp;
#endif
        const uint64_t S = item_start(i), sn = slot_src(S);
        dma_item(slot, sn, lane, item_need(S, sn));
    };
    // this lane's window of item i, realigned and front-masked (d: 25 raw dwords from the slot)
    auto read_window = [&](const uint8_t *slot, uint64_t i, uint32_t (&d)[kChunkWords + 1]) -> uint32_t {
        const uint64_t S = item_start(i), src = slot_src(S);
        const int64_t x = (int64_t)(S - src) + klane;   // window start within the slot (>= -28)
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(slot + (x & ~3ll));
#pragma unroll
        for (int q = 0; q < kChunkWords; q++) d[q] = wp[q];
        // the 25th dword matters only when r != 0; then it lies inside the slot. Clamped so the
        // last slot in LDS is never read past its end.
        const uint64_t a24 = (uint64_t)(wp + kChunkWords), lim = (uint64_t)(slot + kDmaItemBytes - 4);
        d[kChunkWords] = *reinterpret_cast<const uint32_t *>(a24 < lim ? a24 : lim);
        return (uint32_t)x & 3u;
    };
    auto realign = [&](const uint32_t (&d)[kChunkWords + 1], uint32_t r, uint32_t (&w)[kChunkWords]) {
#pragma unroll
        for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], r);
#pragma unroll
        for (int i = 0; i < MW; i++) w[i] &= m[i];
    };

    if constexpr (kDmaPair) {
        // ---- two items per wave at once (8 waves per CU, one slot each): half the DMA streams
        //      of 16 one-slot waves with the same bytes in flight, and both items' chains
        //      interleaved (2 kDmaChains independent chains per lane) ----
        const uint8_t *slot1 = slot0 + kDmaItemBytes;
        uint64_t ia = D.first();
        uint64_t ib = ia != kEnd ? D.next(ia) : kEnd;
        if (ia != kEnd) dma_of(slot0, ia);
        if (ib != kEnd) dma_of(slot1, ib);
        while (ia != kEnd) {   // wave-uniform
            const bool hb = ib != kEnd;
            uint32_t da[kChunkWords + 1], db[kChunkWords + 1];
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): both slots have landed
            const uint32_t ra = read_window(slot0, ia, da);
            const uint32_t rb = read_window(slot1, hb ? ib : ia, db);
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): both slots are free for the next DMAs
            uint64_t na = kEnd, nb = kEnd;
            if (hb) {
                na = D.next(ib);
                if (na != kEnd) nb = D.next(na);
            }
            if (na != kEnd) dma_of(slot0, na);
            if (nb != kEnd) dma_of(slot1, nb);
            if (STREAM) {
                uint32_t acc = ra ^ rb;
#pragma unroll
                for (int q = 0; q <= kChunkWords; q++) acc ^= da[q] ^ db[q];
                if (acc == 0x9E3779B9u) p.out[0] = acc;   // keeps the reads live; practically never stores
            } else {
                uint32_t wa[kChunkWords], wb[kChunkWords];
                realign(da, ra, wa);
                realign(db, rb, wb);
                constexpr int CL = kDmaChainWords;
                uint32_t xa[kDmaChains], xb[kDmaChains];
#pragma unroll
                for (int hh = 0; hh < kDmaChains; hh++) {
                    xa[hh] = wa[hh * CL] ^ (hh == 0 ? x0 : 0u);
                    xb[hh] = wb[hh * CL] ^ (hh == 0 ? x0 : 0u);
                }
#pragma unroll
                for (int i = 0; i < CL; i++)
#pragma unroll
                    for (int hh = 0; hh < kDmaChains; hh++) {
                        xa[hh] = step4_l8(lds, xa[hh], i < CL - 1 ? wa[hh * CL + i + 1] : 0u, B, SEL);
                        xb[hh] = step4_l8(lds, xb[hh], i < CL - 1 ? wb[hh * CL + i + 1] : 0u, B, SEL);
                    }
                uint32_t ma = xa[kDmaChains - 1], mb = xb[kDmaChains - 1];
#pragma unroll
                for (int hh = 0; hh < kDmaChains - 1; hh++) {
                    ma = merge_shift_dma(lds, kDmaChains - 2 - hh, xa[hh], ma);
                    mb = merge_shift_dma(lds, kDmaChains - 2 - hh, xb[hh], mb);
                }
                const uint32_t va = row_xor(lane_shift_dma(lds, ma, lanebase));
                const uint32_t vb = row_xor(lane_shift_dma(lds, mb, lanebase));
                emit<kDmaBad>(p, lds, c == kGroup - 1 && 4 * ia + g < p.n, 4 * ia + g, ~va);
                emit<kDmaBad>(p, lds, hb && c == kGroup - 1 && 4 * ib + g < p.n, 4 * ib + g, ~vb);
            }
            ia = na;
            ib = nb;
        }
        flush_bad<kDmaBad>(p, lds);
        return;
    }

    uint64_t it = D.first();
    if (it != kEnd) dma_of(slot0, it);

#ifdef FCS_STAMPS   // measurement-only: per-wave cycles waiting for the slot vs. the whole item
    uint64_t st_wait = 0, st_all = 0, st_items = 0;
    const uint64_t st_rt0 = __builtin_amdgcn_s_memrealtime(), st_c0 = __builtin_amdgcn_s_memtime();
#endif
    while (it != kEnd) {   // wave-uniform
        const uint8_t *slot = slot0;
        const uint64_t f = 4 * it;
        const uint64_t S = item_start(it);
        const uint64_t src = slot_src(S);
#ifdef FCS_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
#endif
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's slot DMA has landed
#ifdef FCS_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t ts1 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        st_wait += ts1 - ts0;
#endif
        const int64_t x = (int64_t)(S - src) + klane;   // window start within the slot (>= -28)
        const uint32_t r = (uint32_t)x & 3u;
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(slot + (x & ~3ll));
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int q = 0; q < kChunkWords; q++) d[q] = wp[q];
        {   // the 25th dword matters only when r != 0; then it lies inside the slot. Clamped so the
            // last slot in LDS is never read past its end.
            const uint64_t a24 = (uint64_t)(wp + kChunkWords), lim = (uint64_t)(slot + kDmaItemBytes - 4);
            d[kChunkWords] = *reinterpret_cast<const uint32_t *>(a24 < lim ? a24 : lim);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next DMA
        const uint64_t nxt = D.next(it);
        if (nxt != kEnd) dma_of(slot, nxt);

        if (STREAM) {   // read ceiling: the words are only XORed together
            uint32_t acc = r;
#pragma unroll
            for (int q = 0; q <= kChunkWords; q++) acc ^= d[q];
            if (acc == 0x9E3779B9u) p.out[0] = acc;   // keeps the reads live; practically never stores
            it = nxt;
#ifdef FCS_STAMPS
            st_all += __builtin_amdgcn_s_memtime() - ts0;
            st_items++;
#endif
            continue;
        }
        uint32_t w[kChunkWords];
#pragma unroll
#ifdef FCS_DMA_ABL_NOALIGN   // measurement-only: no realignment (wrong FCS unless r == 0)
        for (int i = 0; i < kChunkWords; i++) w[i] = d[i] ^ (i == 0 ? r : 0u);
#else
        for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], r);
#endif
#pragma unroll
        for (int i = 0; i < MW; i++) w[i] &= m[i];
        // kDmaChains independent chains of CL words; chain h ends 4 CL (kDmaChains - 1 - h) bytes
        // before the window end, so the window value is XOR_h A_{4 CL (kDmaChains - 1 - h)}(chain h)
        constexpr int CL = kDmaChainWords;
        uint32_t xs[kDmaChains];
#pragma unroll
        for (int hh = 0; hh < kDmaChains; hh++) xs[hh] = w[hh * CL] ^ (hh == 0 ? x0 : 0u);
#pragma unroll
        for (int i = 0; i < CL; i++)
#pragma unroll
            for (int hh = 0; hh < kDmaChains; hh++)
                xs[hh] = step4_l8(lds, xs[hh], i < CL - 1 ? w[hh * CL + i + 1] : 0u, B, SEL);
        uint32_t mv = xs[kDmaChains - 1];
#pragma unroll
        for (int hh = 0; hh < kDmaChains - 1; hh++) mv = merge_shift_dma(lds, kDmaChains - 2 - hh, xs[hh], mv);
        uint32_t v = lane_shift_dma(lds, mv, lanebase);
        v = row_xor(v);
        emit<kDmaBad>(p, lds, c == kGroup - 1 && f + g < p.n, f + g, ~v);
        it = nxt;
#ifdef FCS_STAMPS
        __builtin_amdgcn_sched_barrier(0);
        st_all += __builtin_amdgcn_s_memtime() - ts0;
        st_items++;
        __builtin_amdgcn_sched_barrier(0);
#endif
    }
#ifdef FCS_STAMPS
    if (p.dbg != nullptr && lane == 0) {
        const uint32_t wv = blockIdx.x * kDmaWaves + (uint32_t)wave;
        p.dbg[wv * 8 + 0] = st_wait;
        p.dbg[wv * 8 + 1] = st_all;
        p.dbg[wv * 8 + 2] = st_items;
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        p.dbg[wv * 8 + 3] = rt1 - st_rt0;
        p.dbg[wv * 8 + 4] = __builtin_amdgcn_s_memtime() - st_c0;
        p.dbg[wv * 8 + 5] = st_rt0;
        p.dbg[wv * 8 + 6] = rt1;
        p.dbg[wv * 8 + 7] = __builtin_amdgcn_s_getreg(/*HW_REG_XCC_ID*/ (20 << 0) | (0 << 6) | (3 << 11));
    }
#endif
    flush_bad<kDmaBad>(p, lds);
}

#ifdef FCS_DMASEG
// ---------------------------------------------------------------------------------------------
// MEASUREMENT-ONLY (-DFCS_DMASEG -DFCS_NO_SEGIL; superseded by fcs_segil_kernel below, DESIGN.md
// §3.2c). Fixed length over 1524 B (jumbo frames, e.g. 9000 B), staged through LDS by DMA
// (fcs_dmaseg_kernel; selected by fixed_dmaseg(): packed frames, stride - len <= 8, and a
// split into m = ceil(len / 1524) segments of Ls = floor(len / m) >= 1496 bytes, the front one
// Lf = Ls + len mod m <= 1524 bytes).
// Every segment is then shaped like a frame of fcs_dma_kernel: its 16 lane windows end e_c bytes
// before the segment end, and only lane 15 masks the 1524 - Ls (front: 1524 - Lf) cover bytes
// before the segment start (loop-invariant masks); the front segment's lane 15 injects INV. The
// frame's register is XOR_s A_{Ls s}(v_s), s = 0 for the frame's last segment.
// The segments of a unit of F frames (F m a multiple of 4, F = 1, 2 or 4) form a stream; a wave's
// item is 4 consecutive stream segments, one per quarter-wave, in one 6 KiB slot DMA (consecutive
// segments of packed frames are contiguous). Quarter q places its segment value in its frame with
// one table shift, A_{Ls s} (the place tables for s = 1 .. m - 1: s <= 4 from the blob, the rest
// composed at staging); a frame's register is then the plain XOR of its placed segments, summed
// over the items by wave-uniform code on the four quarter values (the frame open at the item start
// carries its partial XOR C). Units come from the dispenser, so a frame's segments are all
// processed by one wave, in order.
// An earlier form advanced each quarter only over the segments of its frame that follow in the
// item (A_{Ls t}, t <= 3) and the carried register by A_{Ls k}: a second table shift per item,
// 1.7 % slower at 9000 B.
// A first version cut frames into 1524-B segments from the frame end (one short front segment,
// lanes above its first byte zeroed, a partial lane masked per item): the per-item mask code
// broke the chain block's scheduling and ran 2-12 % slower than the register-load kernel.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kDmaSegJumpHole = kDmaInvHole + 4;   // 4 holes per table: A_{Ls k}, k = 1 .. m - 1
static_assert(kDmaSegJumpHole + 4 * (kDmaSegMaxSegs - 1) <= 256, "place tables overrun the table holes");
static_assert(FCS_DMASEG_MAX_SEGS <= kDmaSegMaxSegs, "segment limit");

// A_{Ls k}(s) for k = 1 .. m - 1; k = 0 returns s. Nibble table t of A_{Ls k} at hole
// kDmaSegJumpHole + 4 (k - 1) + t / 2, +64 B for odd t.
__device__ __forceinline__ uint32_t seg_jump(const uint8_t *lds, uint32_t k, uint32_t s) {
    uint32_t r[8];
    const uint32_t kk = k ? k - 1u : 0u;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        const uint32_t base = dma_hole(kDmaSegJumpHole + 4u * kk + (uint32_t)(t >> 1)) + 64u * (uint32_t)(t & 1);
        r[t] = lds_rd(lds, (sh & 0x3Cu) | base);
    }
    const uint32_t v = xor9(r, 0u);
    return k ? v : s;
}

// MW: words lane 15's masks can touch (host-selected: 2 when 1524 - Lf <= 8, else kSingleMaskWords).
template <int MW>
__global__ __launch_bounds__(kDmaWgThreads, 1) void fcs_dmaseg_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDmaLdsBytes];
    const int tid = threadIdx.x;
    // ---- frame geometry (wave-uniform) ----
    const uint32_t L = p.flen;
    const uint32_t m = (L + kDmaCover - 1) / kDmaCover;                    // segments per frame, >= 2
    const uint32_t F = (m & 3u) == 0 ? 1u : ((m & 1u) == 0 ? 2u : 4u);     // frames per unit
    const uint32_t Ls = L / m, Lf = L - Ls * (m - 1);                        // segment, front segment

    stage_dma_tables(p, lds, tid);
    for (int i = tid; i < 4 * 128; i += kDmaWgThreads) {   // place tables A_{Ls k}, k = 1..4, from the blob
        const int k = i >> 7, t = (i >> 4) & 7, e = i & 15;
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kDmaSegJumpHole + 4u * (uint32_t)k + (uint32_t)(t >> 1)) +
                                      64u * (uint32_t)(t & 1) + 4u * (uint32_t)e) =
            p.blob[kBlobSegJump + (Ls - kDmaMinLen) * 512u + (uint32_t)i];
    }
    // A_{Ls k} for k = 5 .. m - 1: composed here as A_{Ls 4} o A_{Ls (k - 4)}, one k at a time
    for (uint32_t k = 5; k < m; k++) {
        __syncthreads();
        if (tid < 128) {
            const uint32_t t = (uint32_t)tid >> 4, e = (uint32_t)tid & 15u;
            const uint32_t at = 64u * (t & 1u) + 4u * e;
            const uint32_t prev = lds_rd(lds, dma_hole(kDmaSegJumpHole + 4u * (k - 5u) + (t >> 1)) + at);
            const uint32_t v = seg_jump(lds, 4u, prev);
            *reinterpret_cast<uint32_t *>(lds + dma_hole(kDmaSegJumpHole + 4u * (k - 1u) + (t >> 1)) + at) = v;
        }
    }
    init_bad<kDmaBad>(lds);
    __syncthreads();

    const int lane = tid & 63;
    const int c = lane & (kGroup - 1);        // window index back from the segment end
    const uint32_t q = (uint32_t)lane >> 4;   // quarter: stream segment 4 j + q of the item
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint8_t *slot = lds + kDmaRing + (uint32_t)wave * kDmaItemBytes;
    const uint32_t h = (uint32_t)(lane >> 3) & 3u, r4 = (uint32_t)(lane & 7) * 4u;
    const uint32_t B[4] = {r4 + 32u * (0u ^ h), r4 + 32u * (1u ^ h), r4 + 32u * (2u ^ h), r4 + 32u * (3u ^ h)};
    const uint32_t SEL[4] = {0x0C0C0400u + ((0u ^ h) << 8), 0x0C0C0400u + ((1u ^ h) << 8),
                             0x0C0C0400u + ((2u ^ h) << 8), 0x0C0C0400u + ((3u ^ h) << 8)};
    const uint32_t lanebase = kDmaHole + (uint32_t)(lane & 31) * 4u;
    const uint32_t ec = dma_end_off(c);

    // loop invariants: lane 15 masks the cover bytes before its segment (front and other
    // segments), lanes 3/7/11 their overlap word; INV start of the front segment's lane 15
    const int zn = (c == kGroup - 1) ? (int)(kDmaCover - Ls) : (dma_short_lane(c) ? 4 : 0);
    const int zf = (c == kGroup - 1) ? (int)(kDmaCover - Lf) : (dma_short_lane(c) ? 4 : 0);
    static_assert(MW >= 1 && MW <= kSingleMaskWords, "mask words");
    uint32_t mn[MW], mf[MW];
#pragma unroll
    for (int i = 0; i < MW; i++) {
        int t = zn - 4 * i, u = zf - 4 * i;
        t = t < 0 ? 0 : (t > 4 ? 4 : t);
        u = u < 0 ? 0 : (u > 4 ? 4 : u);
        mn[i] = (uint32_t)(0xFFFFFFFFull << (8 * t));
        mf[i] = (uint32_t)(0xFFFFFFFFull << (8 * u));
    }
    const uint32_t x0f = (c == kGroup - 1)
                             ? lds_rd(lds, dma_hole(kDmaInvHole + (uint32_t)zf / 32u) + (uint32_t)(zf % 32) * 4u)
                             : 0u;

    const uint64_t lo16 = p.lo4 & ~15ull;
    const uint64_t smax = ((p.hi4 + 15) & ~15ull) - kDmaItemBytes;   // last slot start inside the arena
    auto slot_src = [&](uint64_t S) {
        const uint64_t a = S & ~15ull;
        return a < lo16 ? lo16 : (a > smax ? smax : a);
    };
    constexpr uint64_t kEnd = Dispenser::kEnd;
    const uint64_t units = (p.n + F - 1) / F;
    const uint32_t per_unit = F * m / 4;                                    // items of a full unit
    const uint32_t cmax = per_unit >= 64 ? 1u : 64u / per_unit;
    Dispenser D(p.ctr, units, (uint64_t)gridDim.x * kDmaWaves, (uint64_t)blockIdx.x * kDmaWaves + (uint64_t)wave,
                lane, 100, 1, cmax);

    // Item state, wave-uniform: unit u (frames u F ..), item j of J, and the stream position of
    // quarter 0: frame fi0 of the unit, segment r0 counted from the frame's front (s = m - 1 - r).
    struct It {
        uint64_t u, fb0, src;   // fb0: start of quarter 0's frame; src: slot start
        uint32_t j, J, Fu, fi0, r0, need;
    };
    auto seg_end = [&](uint32_t r) { return (uint64_t)Lf + (uint64_t)Ls * r; };   // from the frame start
    auto place = [&](It &t) {
        t.fb0 = p.base + (t.u * F + t.fi0) * p.stride;
        t.src = slot_src(t.fb0 + (t.r0 ? seg_end(t.r0 - 1) : 0));
        const uint32_t last = 4 * t.j + 3 < t.Fu * m ? 3u : t.Fu * m - 1u - 4 * t.j;   // last active quarter
        uint32_t fi = 0, r = t.r0 + last;
        while (r >= m) {
            r -= m;
            fi++;
        }
        const uint64_t nb = t.fb0 + fi * p.stride + seg_end(r) + 4 - t.src;
        t.need = (uint32_t)(nb < (uint64_t)kDmaItemBytes ? nb : (uint64_t)kDmaItemBytes);
    };
    auto start_unit = [&](It &t, uint64_t u) {
        t.u = u;
        t.j = 0;
        t.fi0 = 0;
        t.r0 = 0;
        const uint64_t left = p.n - u * F;
        t.Fu = left < F ? (uint32_t)left : F;
        t.J = (t.Fu * m + 3u) / 4u;
        place(t);
    };

    It cur{};
    bool live = false;
    {
        const uint64_t u0 = D.first();
        if (u0 != kEnd) {
            start_unit(cur, u0);
            live = true;
            dma_item<true>(slot, cur.src, lane, cur.need);
        }
    }
    uint32_t C = 0;   // register of the frame open at the item start (wave-uniform)
    while (live) {
        // this lane's segment: quarter q = stream position (fi0, r0) + q
        uint32_t dfi = 0, r = cur.r0 + q;
        while (r >= m) {
            r -= m;
            dfi++;
        }
        const bool act = cur.fi0 + dfi < cur.Fu;
        const uint32_t s = m - 1u - r;
        const bool front = r == 0;
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's slot DMA has landed
        const int64_t x = act ? (int64_t)(cur.fb0 + dfi * p.stride + seg_end(r) - cur.src) - (int64_t)ec - kChunkBytes : 0;
        const uint32_t ra = (uint32_t)x & 3u;
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(slot + (x & ~3ll));
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int i = 0; i < kChunkWords; i++) d[i] = wp[i];
        {
            const uint64_t a24 = (uint64_t)(wp + kChunkWords), lim = (uint64_t)(slot + kDmaItemBytes - 4);
            d[kChunkWords] = *reinterpret_cast<const uint32_t *>(a24 < lim ? a24 : lim);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next DMA

        // ---- the next item (same unit, or the dispenser's next unit): its DMA lands meanwhile ----
        It nxt = cur;
        bool nlive = true;
        if (cur.j + 1 < cur.J) {
            nxt.j++;
            nxt.r0 += 4;
            while (nxt.r0 >= m) {
                nxt.r0 -= m;
                nxt.fi0++;
            }
            place(nxt);
        } else {
            const uint64_t un = D.next(cur.u);
            nlive = un != kEnd;
            if (nlive) start_unit(nxt, un);
        }
        if (nlive) dma_item<true>(slot, nxt.src, lane, nxt.need);

        // ---- this item's segment values ----
        uint32_t w[kChunkWords];
#pragma unroll
        for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], ra);
#pragma unroll
        for (int i = 0; i < MW; i++) w[i] &= front ? mf[i] : mn[i];
        constexpr int CL = kDmaChainWords;
        uint32_t xs[kDmaChains];
#pragma unroll
        for (int hh = 0; hh < kDmaChains; hh++) xs[hh] = w[hh * CL] ^ (hh == 0 && front ? x0f : 0u);
#pragma unroll
        for (int i = 0; i < CL; i++)
#pragma unroll
            for (int hh = 0; hh < kDmaChains; hh++)
                xs[hh] = step4_l8(lds, xs[hh], i < CL - 1 ? w[hh * CL + i + 1] : 0u, B, SEL);
        uint32_t mv = xs[kDmaChains - 1];
#pragma unroll
        for (int hh = 0; hh < kDmaChains - 1; hh++) mv = merge_shift_dma(lds, kDmaChains - 2 - hh, xs[hh], mv);
        uint32_t v = lane_shift_dma(lds, mv, lanebase);
        v = act ? v : 0u;
        v = row_xor(v);
        // placed in its frame: A_{Ls s}, s segments before the frame end
#ifdef FCS_SEG_ABL_NOJUMP   // measurement-only: no placement shift (wrong FCS)
        const uint32_t uq = v ^ s;
#else
        const uint32_t uq = seg_jump(lds, act ? s : 0u, v);
#endif

#ifdef FCS_SEG_ABL_NOCOMB   // measurement-only: each quarter's value stored as is (wrong FCS)
        emit<kDmaBad>(p, lds, c == 0 && act, cur.u * F + cur.fi0 + dfi, ~uq);
        cur = nxt;
        live = nlive;
        continue;
#endif
        // ---- per-frame accumulation (wave-uniform) ----
        uint32_t acc = 0;
        if (cur.r0 != 0) acc = C;   // the frame open at the item start: its placed segments so far
        uint32_t rq = cur.r0, fq = cur.fi0;
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            if (fq >= cur.Fu) break;
            const uint32_t vq = (uint32_t)__builtin_amdgcn_readlane((int)uq, 16 * qq);
            acc = rq == 0 ? vq : (acc ^ vq);
            if (rq == m - 1u) emit<kDmaBad>(p, lds, lane == 0, cur.u * F + fq, ~acc);
            if (++rq == m) {
                rq = 0;
                fq++;
            }
        }
        C = acc;

        cur = nxt;
        live = nlive;
    }
    flush_bad<kDmaBad>(p, lds);
}
#endif  // FCS_DMASEG

// ---------------------------------------------------------------------------------------------
// Fixed length over 1524 B, any stride: frame-interleaved segments staged through LDS by DMA
// (fcs_segil_kernel; host-selected by fixed_segil()).
// A frame of L bytes is cut from its front into m = ceil(L / 1524) segments: a front segment of
// Lf = L - 1524 (m - 1) bytes, then m - 1 segments of exactly 1524 bytes. A wave's unit is four
// frames, one per quarter-wave; item r of a unit is segment r of its four frames: four runs of at
// most 97 16-B pieces (the segment plus the alignment of its ends), each DMAed into its own 2 KiB
// part of the wave's 8 KiB slot (two rows: 64 + 33 lanes). A 1524-B segment is exactly the cover
// of fcs_dma_kernel's 16 lane windows, so it needs no mask beyond the short lanes' overlap word,
// and the frame's CRC state after the previous segment enters through lane 15's chain start (a CRC
// state is the same as XORing it into the next four data bytes). No shift is needed between
// segments: the quarter's row XOR after segment r is its frame's CRC state after that segment,
// and stays in a register until the next item. The front item (1 in m) masks each lane's bytes
// before the frame start (loop-invariant per lane: Lf is fixed), drops lanes wholly before it and
// injects INV at the frame's first byte.
// LDS: the 64 KiB table image of fcs_dma_kernel, then 12 slots of 8 KiB (160 KiB).
// ---------------------------------------------------------------------------------------------
constexpr int kSegilWaves = 12;
constexpr int kSegilThreads = kSegilWgThreads;
static_assert(kSegilThreads == 64 * kSegilWaves, "12 waves");
constexpr uint32_t kSegilRunBytes = 2048;                      // one run's part of a slot
constexpr uint32_t kSegilSlotBytes = 4 * kSegilRunBytes;
constexpr uint32_t kSegilLdsBytes = kDmaRing + (uint32_t)kSegilWaves * kSegilSlotBytes;
static_assert(kSegilLdsBytes <= 163840, "LDS per CU");
static_assert(kSegilWaves <= 16, "verify counters: 16 waves");
#ifndef FCS_SEGIL_TAIL_AUX   // cache policy of a run's second row (it holds the line the next segment shares)
#define FCS_SEGIL_TAIL_AUX 0
#endif
#ifndef FCS_SEGIL_SKEW   // bytes added to odd runs' LDS base (bank phase of their windows)
#define FCS_SEGIL_SKEW 16
#endif

// One run's DMA: pieces 0..63 in row 0 (non-temporal), 64..need-1 in row 1.
__device__ __forceinline__ void segil_run(const uint8_t *dst, uint64_t src, int lane, uint32_t pieces) {
    typedef __attribute__((address_space(3))) void lds_void;
    const uint64_t a = src + 16 * (uint64_t)lane;
    lds_void *l = (lds_void *)dst;
    if ((uint32_t)lane < pieces) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), l, 16, 0, FCS_DMA_AUX);
    if ((uint32_t)lane + 64u < pieces)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), l, 16, 1024, FCS_SEGIL_TAIL_AUX);
}

__global__ __launch_bounds__(kSegilThreads, 1) void fcs_segil_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kSegilLdsBytes];
    const int tid = threadIdx.x;
    stage_dma_tables<kSegilThreads>(p, lds, tid);
    init_bad<kDmaBad>(lds);
    __syncthreads();

    // ---- frame geometry (wave-uniform) ----
    const uint32_t L = p.flen;
    const uint32_t m = (L + kDmaCover - 1) / kDmaCover;   // segments, >= 2
    const uint32_t Lf = L - kDmaCover * (m - 1);          // front segment, 1 .. 1524

    const int lane = tid & 63;
    const int c = lane & (kGroup - 1);        // window index back from the segment end
    const uint32_t q = (uint32_t)lane >> 4;   // quarter: frame 4 u + q of unit u
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint8_t *slot = lds + kDmaRing + (uint32_t)wave * kSegilSlotBytes;
    const uint8_t *run = slot + q * kSegilRunBytes + (q & 1u) * FCS_SEGIL_SKEW;
    const uint32_t h = (uint32_t)(lane >> 3) & 3u, r4 = (uint32_t)(lane & 7) * 4u;
    const uint32_t B[4] = {r4 + 32u * (0u ^ h), r4 + 32u * (1u ^ h), r4 + 32u * (2u ^ h), r4 + 32u * (3u ^ h)};
    const uint32_t SEL[4] = {0x0C0C0400u + ((0u ^ h) << 8), 0x0C0C0400u + ((1u ^ h) << 8),
                             0x0C0C0400u + ((2u ^ h) << 8), 0x0C0C0400u + ((3u ^ h) << 8)};
    const uint32_t lanebase = kDmaHole + (uint32_t)(lane & 31) * 4u;
    const uint32_t ec = dma_end_off(c);

    // loop invariants. Other segments: the short lanes' overlap word. Front segment: zr bytes of
    // the lane's window lie before the frame start (>= 96: the whole window, the lane is dropped);
    // the lane holding the first byte in its unmasked part starts its chain from INV there.
    const uint32_t mn0 = dma_short_lane(c) ? 0u : 0xFFFFFFFFu;
    const int zr = (int)(kDmaCover - Lf) - (int)(kDmaCover - ec - kChunkBytes);
    const bool fdead = zr >= kChunkBytes;
    int zf = zr < 0 ? 0 : (zr > kChunkBytes ? kChunkBytes : zr);
    if (dma_short_lane(c) && zf < 4) zf = 4;
    const uint32_t x0f = (!fdead && zr >= 0 && zf == zr)
                             ? lds_rd(lds, dma_hole(kDmaInvHole + (uint32_t)zr / 32u) + (uint32_t)(zr % 32) * 4u)
                             : 0u;
    const int zb = fdead ? 0 : zf;   // the wave masks word groups up to its largest live claim

    const uint64_t n = p.n, units = (n + 3) >> 2;
    const uint32_t cmax = m >= 64 ? 1u : 64u / m;
    Dispenser D(p.ctr, units, (uint64_t)gridDim.x * kSegilWaves, (uint64_t)blockIdx.x * kSegilWaves + (uint64_t)wave,
                lane, 100, 1, cmax);
    constexpr uint64_t kEnd = Dispenser::kEnd;
    // segment r of frame f: [start, start + len); the run starts at the 16-B boundary below it
    auto seg_start = [&](uint64_t f, uint32_t r) {
        return p.base + f * p.stride + (r ? (uint64_t)Lf + (uint64_t)kDmaCover * (r - 1) : 0ull);
    };
    auto issue = [&](uint64_t u, uint32_t r) {   // the item's four runs (wave-uniform control)
        const uint32_t len = r ? kDmaCover : Lf;
#pragma unroll
        for (uint32_t qq = 0; qq < 4; qq++) {
            const uint64_t f = 4 * u + qq;
            if (f < n) {
                const uint64_t s0 = seg_start(f, r), a = s0 & ~15ull;
                const uint32_t pieces = (uint32_t)((((s0 + len) + 15) & ~15ull) - a) >> 4;
                segil_run(slot + qq * kSegilRunBytes + (qq & 1u) * FCS_SEGIL_SKEW, a, lane, pieces);
            }
        }
    };

    uint64_t u = D.first();
    uint32_t r = 0;
    if (u != kEnd) issue(u, 0);
    uint32_t acc = 0;   // this quarter's frame: CRC state after its segments so far
    while (u != kEnd) {   // wave-uniform
        const uint64_t f = 4 * u + q;
        const bool act = f < n;
        const uint64_t s0 = act ? seg_start(f, r) : 0ull;
        const uint32_t len = r ? kDmaCover : Lf;
        const int64_t x = (int64_t)(s0 & 15ull) + (int64_t)len - (int64_t)ec - kChunkBytes;   // window start in the run
        const uint32_t ra = (uint32_t)x & 3u;
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's runs have landed
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(run + (x & ~3ll));
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int i = 0; i <= kChunkWords; i++) d[i] = wp[i];
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next DMA

        // ---- the next item: the next segment of the unit, or the dispenser's next unit ----
        uint64_t un = u;
        uint32_t rn = r + 1;
        if (rn == m) {
            un = D.next(u);
            rn = 0;
        }
        if (un != kEnd) issue(un, rn);

        // ---- this item ----
        uint32_t w[kChunkWords];
#pragma unroll
        for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], ra);
        uint32_t x0;
        if (r == 0) {
            const int zf8 = 8 * zf;
#pragma unroll
            for (int g = 0; g < kChunkWords / 4; g++) {
                if (!__any(zb > 16 * g)) break;
#pragma unroll
                for (int i = 4 * g; i < 4 * g + 4; i++) {
                    // zf is a loop invariant: the compiler hoists this clamp (no v_med3 asm here)
                    int t = zf8 - 32 * i;
                    t = t < 0 ? 0 : (t > 32 ? 32 : t);
                    w[i] &= (uint32_t)(0xFFFFFFFFull << t);
                }
            }
            x0 = x0f;
        } else {
            w[0] &= mn0;
            x0 = c == kGroup - 1 ? acc : 0u;
        }
        constexpr int CL = kDmaChainWords;
        uint32_t xs[kDmaChains];
#pragma unroll
        for (int hh = 0; hh < kDmaChains; hh++) xs[hh] = w[hh * CL] ^ (hh == 0 ? x0 : 0u);
#pragma unroll
        for (int i = 0; i < CL; i++)
#pragma unroll
            for (int hh = 0; hh < kDmaChains; hh++)
                xs[hh] = step4_l8(lds, xs[hh], i < CL - 1 ? w[hh * CL + i + 1] : 0u, B, SEL);
        uint32_t mv = xs[kDmaChains - 1];
#pragma unroll
        for (int hh = 0; hh < kDmaChains - 1; hh++) mv = merge_shift_dma(lds, kDmaChains - 2 - hh, xs[hh], mv);
        uint32_t v = lane_shift_dma(lds, mv, lanebase);
        if (r == 0 && fdead) v = 0u;
        acc = row_xor(v);
        if (r == m - 1) emit<kDmaBad>(p, lds, c == kGroup - 1 && act, f, ~acc);
        u = un;
        r = rn;
    }
    flush_bad<kDmaBad>(p, lds);
}

// ---------------------------------------------------------------------------------------------
// Variable-length frames (IMIX-shaped batches): windowed class scheduling. Superseded by
// fcs_flat_kernel below (+16 % on IMIX); kept as the measurement baseline (-DFCS_VAR_HALFUNIT).
// A wave owns windows of 64 consecutive frames (frame i of a window <-> lane i for metadata).
// The window's frames are split by length into classes that use lanes differently:
//   small  (len <= 96):  the owning lane alone processes the frame as one chunk (chunk 0, no
//                        lane shift, no reduction);
//   medium (len <= 768): 8 lanes per frame (chunk c <- lane & 7), 8 frames per item; lanes 8..15
//                        of a row used the lane tables of chunks 8..15, fixed by one A_{-768};
//   big    (len > 768):  16 lanes per frame (as the fixed kernels), 4 frames per item,
//                        1536-B segments accumulated with A_1536.
// All classes read the same ~64 frames of the arena close together in time (L2-local).
// ---------------------------------------------------------------------------------------------
template <bool TINY>
__device__ __forceinline__ void issue_any(const KParams &p, int64_t cstart, bool need, Chunk &c) {
    LoadPriority lp;
    c.r = (uint32_t)cstart & 3u;
    const uint64_t a = need ? ((uint64_t)cstart & ~3ull) : p.lo4;
    c.dlead = 0;
    if (TINY) {
        uint32_t d[kChunkWords + 1];
#pragma unroll
        for (int q = 0; q <= kChunkWords; q++) {
            const uint64_t ad = a + 4 * q;
            d[q] = (need && ad >= p.lo4 && ad + 4 <= p.hi4) ? gload<uint32_t>(ad) : 0u;
        }
#pragma unroll
        for (int g = 0; g < 6; g++) c.x[g] = u32x4a4{d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]};
        c.x6 = d[kChunkWords];
        return;
    }
    uint64_t ab = a;
    if (__any(a < p.lo4)) {
        c.dlead = a < p.lo4 ? (int)((p.lo4 - a) >> 2) : 0;
        ab = a < p.lo4 ? p.lo4 : a;
    }
#pragma unroll
    for (int q = 0; q < 6; q++) c.x[q] = gload<u32x4a4>(ab + 16 * q);
    c.x6 = gload<uint32_t>(ab + ((c.r || c.dlead) ? 96 : 92));
}

// Register value of one chunk (realigned, bytes before the frame start masked, x0 injected),
// before the lane shift: A_48(chain(words 0..11)) ^ chain(words 12..23).
// zb: this lane's claim on the masking (zr if its value is used, 0 if the caller discards it): the
// wave masks 16-byte groups of words only up to its largest claim (IMIX items: 32 bytes, not 96).
template <bool TINY>
__device__ __forceinline__ uint32_t chunk_value(const uint8_t *lds, const Chunk &c, int zr, int zb, uint32_t x0,
                                                uint32_t base0, uint32_t base1) {
    uint32_t d[kChunkWords + 1];
#pragma unroll
    for (int q = 0; q < 6; q++) {
        d[4 * q] = c.x[q].x;
        d[4 * q + 1] = c.x[q].y;
        d[4 * q + 2] = c.x[q].z;
        d[4 * q + 3] = c.x[q].w;
    }
    d[kChunkWords] = c.x6;
    if (!TINY && __any(c.dlead)) shift_up(d, c.dlead);
    uint32_t w[kChunkWords];
#pragma unroll
    for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], c.r);
#ifdef FCS_MASK_ALL   // measurement-only build: every word masked whenever any lane has a front
    if (__any(zr > 0)) {
#pragma unroll
        for (int i = 0; i < kChunkWords; i++) {
            int t = zr - 4 * i;
            t = t < 0 ? 0 : (t > 4 ? 4 : t);
            w[i] &= (uint32_t)(0xFFFFFFFFull << (8 * t));
        }
    }
#else
    const int zr8 = 8 * zr;
#pragma unroll
    for (int g = 0; g < kChunkWords / 4; g++) {
        if (!__any(zb > 16 * g)) break;
#pragma unroll
        for (int i = 4 * g; i < 4 * g + 4; i++) {
            w[i] = clear_low_bits(w[i], zr8 - 32 * i);
        }
    }
#endif
    uint32_t xa = x0 ^ w[0], xb = w[12];
#pragma unroll
    for (int i = 0; i < 12; i++) {
        xa = step4(lds, xa, i < 11 ? w[i + 1] : 0u, base0, base1);
        xb = step4(lds, xb, i < 11 ? w[13 + i] : 0u, base0, base1);
    }
    return uniform_shift<kLdsH48>(lds, xa, xb);
}

__device__ __forceinline__ uint32_t inv_start(const uint8_t *lds, int zr) {
    const int zi = zr < 0 ? 0 : (zr > kChunkBytes - 1 ? kChunkBytes - 1 : zr);
    const uint32_t iv = lds_rd(lds, kLdsInv + 4u * (uint32_t)zi);
    return (zr >= 0 && zr < kChunkBytes) ? iv : 0u;
}

__device__ __forceinline__ int clamp_zr(int64_t z) {
    return z < -1 ? -1 : (z > kChunkBytes ? kChunkBytes : (int)z);
}

// One half-unit item of the windowed var kernel (fcs_var_kernel): 8 half-units of 8 lanes.
// unit_issue resolves this lane's frame and chunk and issues its loads; unit_finish computes the
// chunk, reduces each frame's lanes and stores.
struct UnitItem {
    Chunk ch;
    uint32_t meta;   // zr + 1 (bits 0-7) | valid (8) | full row (9) | small lane (10) | empty frame (11) |
                     // window lane of this lane's frame (16-21)
};

template <bool TINY>
__device__ __forceinline__ void unit_issue(const KParams &p, const uint8_t *lists, uint32_t Ehi, uint32_t Elo,
                                           uint32_t L, uint32_t nf, uint32_t nfm, uint32_t nu, uint32_t ns,
                                           uint32_t t, int lane, int j, UnitItem &it) {
    const uint32_t u = t + (uint32_t)(lane >> 3);
    const bool isfull = u < 2 * nf;   // same for both halves of a row
    const bool issmall = u >= nfm;
    const uint32_t si = (u - nfm) * 8 + (uint32_t)(lane & 7);   // small frame rank
    const bool valid = issmall ? (u < nu && si < ns) : u < nu;
    const int src = valid ? (int)lists[isfull ? 64 + (u >> 1) : (issmall ? 192 + si : u - 2 * nf)] : 0;
    const uint64_t Eg = ((uint64_t)(uint32_t)__shfl((int)Ehi, src) << 32) | (uint32_t)__shfl((int)Elo, src);
    const uint32_t Lg = (uint32_t)__shfl((int)L, src);
    const int c = isfull ? j : (issmall ? 0 : (lane & 7));   // chunk index back from the frame end
    const int64_t cstart = (int64_t)Eg - (int64_t)kChunkBytes * (c + 1);
    const int zr = clamp_zr((int64_t)(Eg - Lg) - cstart);
    issue_any<TINY>(p, cstart, valid && zr < kChunkBytes, it.ch);
    it.meta = (uint32_t)((valid ? zr : kChunkBytes) + 1) | (valid ? 1u << 8 : 0u) | (isfull ? 1u << 9 : 0u) |
              (issmall ? 1u << 10 : 0u) | (Lg == 0 ? 1u << 11 : 0u) | ((uint32_t)src << 16);
}

template <bool TINY>
__device__ __forceinline__ void unit_finish(const KParams &p, const uint8_t *lds, const UnitItem &it, uint64_t w0,
                                            int lane, int j, uint32_t base0, uint32_t base1, uint32_t lanebase) {
    const bool valid = it.meta & (1u << 8), isfull = it.meta & (1u << 9), issmall = it.meta & (1u << 10);
    const int zr = (int)(it.meta & 0xFFu) - 1;
    const uint32_t own = chunk_value<TINY>(lds, it.ch, zr, zr, valid ? inv_start(lds, zr) : 0u, base0, base1);
    uint32_t v = lane_shift(lds, own, lanebase);   // A_{96 j}
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // half_mirror
    // full rows join their halves (row_mirror); medium upper halves used A_{96(c+8)}: undo A_768
    const uint32_t joined = v ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    const uint32_t fixed = uniform_shift<kLdsM768>(lds, v, 0u);
    v = isfull ? joined : (issmall ? own : (j >= 8 ? fixed : v));
    emit(p, lds, valid && (isfull ? j == 15 : (issmall || (lane & 7) == 7)), w0 + ((it.meta >> 16) & 63u),
         (it.meta & (1u << 11)) ? 0u : ~v);
}

template <bool TINY>
__global__ __launch_bounds__(kWgThreads, 1) void fcs_var_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    stage_tables<kWgThreads>(p, lds);
    init_bad(lds);

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int j = lane & (kGroup - 1);
    const uint32_t r4 = (uint32_t)(lane & 31) * 4u;
    const uint32_t lanebase = kLdsLane | r4;
    uint32_t base0, base1;
    table_bases(lane, base0, base1);
    uint8_t *lists = lds + kLdsWave + wave * kLdsWaveBytes;   // medium | full | multi | small, 64 each
    const uint64_t GW = (uint64_t)gridDim.x * (kWgThreads / 64);

    for (uint64_t w0 = ((uint64_t)blockIdx.x * (kWgThreads / 64) + wave) * 64; w0 < p.n; w0 += GW * 64) {
        // ---- window metadata: lane i <-> frame w0 + i ----
        const uint64_t f = w0 + lane;
        const bool act = f < p.n;
        const uint32_t L = act ? (p.len ? p.len[f] : p.flen) : 0u;   // len == null: fixed length
        const uint64_t E = act ? p.base + (p.off ? p.off[f] : f * p.stride) + L : p.lo4;   // off == null: slots of p.stride
        const bool small = act && L <= (uint32_t)kChunkBytes;
        const bool med = act && !small && L <= 8u * kChunkBytes;
        const bool full = act && L > 8u * kChunkBytes && L <= (uint32_t)kSegBytes;
        const bool multi = act && L > (uint32_t)kSegBytes;
        const uint64_t mmask = __ballot(med), fmask = __ballot(full), xmask = __ballot(multi);
        const uint32_t nm = (uint32_t)__popcll(mmask), nf = (uint32_t)__popcll(fmask), nx = (uint32_t)__popcll(xmask);
        const uint32_t rm = __builtin_amdgcn_mbcnt_hi((uint32_t)(mmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mmask, 0u));
        const uint32_t rf = __builtin_amdgcn_mbcnt_hi((uint32_t)(fmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fmask, 0u));
        const uint32_t rx = __builtin_amdgcn_mbcnt_hi((uint32_t)(xmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)xmask, 0u));
        if (med) lists[rm] = (uint8_t)lane;
        if (full) lists[64 + rf] = (uint8_t)lane;
        if (multi) lists[128 + rx] = (uint8_t)lane;
        const uint64_t smask = __ballot(small);
        const uint32_t ns = (uint32_t)__popcll(smask);
        const uint32_t rs = __builtin_amdgcn_mbcnt_hi((uint32_t)(smask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)smask, 0u));
        if (small) lists[192 + rs] = (uint8_t)lane;
        const uint32_t Elo = (uint32_t)E, Ehi = (uint32_t)(E >> 32);

        // ---- half-units (8 lanes each, 8 per item), in this order:
        //      full frame (769..1536 B): two halves of one 16-lane row (chunk index = j);
        //      medium frame (97..768 B): one half (chunk index = lane & 7);
        //      small frames (<= 96 B): eight per half, one lane each, a single chunk.
        //      Full frames come first, so their rows are aligned. ----
        const uint32_t nfm = 2 * nf + nm;
        const uint32_t nu = nfm + (ns + 7) / 8;
        // one item at a time: a second item in flight measured 5-7 % slower here (the var loop is
        // issue-bound, and the extra registers cost waits), unlike the fixed kernels
        for (uint32_t t = 0; t < nu; t += 8) {
            UnitItem A;
            unit_issue<TINY>(p, lists, Ehi, Elo, L, nf, nfm, nu, ns, t, lane, j, A);
            unit_finish<TINY>(p, lds, A, w0, lane, j, base0, base1, lanebase);
        }

        // ---- multi-segment frames (> 1536 B): 16 lanes each, 4 per item, segment by segment ----
        for (uint32_t t = 0; t < nx; t += 4) {
            const uint32_t rank = t + (uint32_t)(lane >> 4);
            const bool valid = rank < nx;
            const int src = valid ? (int)lists[128 + rank] : 0;
            const uint64_t Eq = ((uint64_t)(uint32_t)__shfl((int)Ehi, src) << 32) | (uint32_t)__shfl((int)Elo, src);
            const uint32_t Lq = (uint32_t)__shfl((int)L, src);
            const uint32_t m = valid ? (Lq + (kSegBytes - 1)) / kSegBytes : 0u;
            uint32_t s = 0;
            for (uint32_t k = 0; __any(k < m); k++) {
                const bool on = k < m;
                const int64_t cstart = (int64_t)Eq - (int64_t)kSegBytes * (int64_t)(m - 1 - k) -
                                       (int64_t)kChunkBytes * (j + 1);
                const int zr = (on && k == 0) ? clamp_zr((int64_t)(Eq - Lq) - cstart) : (on ? -1 : kChunkBytes);
                Chunk c;
                issue_any<TINY>(p, cstart, on && zr < kChunkBytes, c);
                const uint32_t r = chunk_value<TINY>(lds, c, zr, on ? zr : 0, (on && k == 0) ? inv_start(lds, zr) : 0u,
                                                     base0, base1);
                s = on ? (k == 0 ? r : uniform_shift<kLdsJump>(lds, s, r)) : s;
            }
            uint32_t v = lane_shift(lds, s, lanebase);
            v = row_xor(v);
            emit(p, lds, valid && j == 15, w0 + (uint32_t)src, Lq ? ~v : 0u);
        }
    }
    flush_bad(p, lds);
}

// ---------------------------------------------------------------------------------------------
// Variable-length frames, flat chunk stream (fcs_flat_kernel).
// A wave owns windows of 64 consecutive frames. Every frame of at most 1536 bytes needs
// k = ceil(len / 96) chunks (an empty frame one dummy chunk); the window's chunks are numbered
// frame by frame (exclusive prefix P over the window) and dealt to the lanes 64 at a time, so
// every lane of an item carries a real chunk whatever the mix of lengths (a 576-B frame takes
// 6 lanes, not 8; small, medium and full frames pack without gaps). Per item a lane finds its
// frame from the frame-start marks (one LDS byte per chunk slot, a ballot and a popcount),
// computes its chunk's register exactly as the other kernels do, shifts it by A_{96c} for its
// chunk index c (tables indexed by c, stride 4 mod 64 banks) and XORs it into the frame's LDS
// accumulator (ds_xor). At the end of the window lane i stores frame i's FCS: one coalesced
// store per window. Frames over 1536 bytes take the segment loop of fcs_var_kernel.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t chunk_shift(const uint8_t *lds, uint32_t s, uint32_t c) {
    uint32_t r[8];
    const uint32_t base = kLdsFlat + c * kFlatStride;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        r[t] = lds_rd(lds, base + (sh & 0x3Cu) + t * 64);
    }
    return xor9(r, 0u);
}

template <bool TINY>
__global__ __launch_bounds__(kWgThreads, 1) void fcs_flat_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    stage_tables_flat(p, lds);
    init_bad(lds);

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int j = lane & (kGroup - 1);
    uint32_t base0, base1;
    table_bases(lane, base0, base1);
    uint32_t *acc = reinterpret_cast<uint32_t *>(lds + kLdsWave + wave * kLdsWaveBytes);   // 64 frames
    uint8_t *mark = lds + kLdsFlatMark + wave * 64;
    uint8_t *list = lds + kLdsFlatList + wave * 64;
    acc[lane] = 0u;
    mark[lane] = 0;
    // windows of 64 frames from the dispenser (dynamic chunks of up to 16 windows when p.ctr is set)
    Dispenser D(p.ctr, (p.n + 63) >> 6, (uint64_t)gridDim.x * (kWgThreads / 64),
                (uint64_t)blockIdx.x * (kWgThreads / 64) + (uint64_t)wave, lane, 100, 1, FCS_FLAT_CHUNK_MAX);
    for (uint64_t win = D.first(); win != Dispenser::kEnd; win = D.next(win)) {
        const uint64_t w0 = win * 64;
        // ---- window metadata: lane i <-> frame w0 + i ----
        const uint64_t f = w0 + lane;
        const bool act = f < p.n;
        const uint32_t L = act ? (p.len ? p.len[f] : p.flen) : 0u;   // len == null: fixed length
        const uint64_t E = act ? p.base + (p.off ? p.off[f] : f * p.stride) + L : p.lo4;
        const bool multi = act && L > (uint32_t)kSegBytes;
        const uint32_t k = (!act || multi) ? 0u : (L ? (L + kChunkBytes - 1) / kChunkBytes : 1u);
        uint32_t incl = k;   // inclusive prefix over the window
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t P = incl - k;
        const uint32_t PL = P | ((L > 0xFFFFu ? 0xFFFFu : L) << 16);   // see deal()
        const uint32_t K = (uint32_t)__shfl((int)incl, 63);
        const uint64_t fmask = __ballot(k != 0);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fmask, 0u));
        if (k) list[rank] = (uint8_t)lane;
        wave_lds_sync();
        const uint32_t Elo = (uint32_t)E, Ehi = (uint32_t)(E >> 32);
#ifndef FCS_FLAT_NO_SHORTCUTS   // measurement-only: always the list read and four bpermutes
        // common windows: no frame over 1536 B (the frames with chunks are lanes 0, 1, ..., so a
        // chunk's frame rank is its frame's lane: no list read), and all frame ends in one 4 GiB
        // page of addresses (the high word is shared: one bpermute fewer)
        const bool dense = __ballot(multi) == 0;
        const uint32_t Ehi0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)Ehi);
        const bool onehi = __ballot(Ehi != Ehi0) == 0;
#else
        const bool dense = false, onehi = false;
        const uint32_t Ehi0 = 0;
#endif

        // one item = 64 chunks; resolve lane -> (frame, chunk) and issue its loads
        struct FlatItem {
            Chunk ch;
            int src, zr;
            uint32_t c;
            bool valid;
            int64_t cstart;
        };
        auto deal = [&](uint32_t g0, uint32_t tag, FlatItem &it) {
            // frame starts inside this item: mark their slot, then lane g finds its frame's rank
            // as (frames started before the item) + (marks at or below g) - 1
            if (k && P >= g0 && P < g0 + 64) mark[P - g0] = (uint8_t)tag;
            wave_lds_sync();
            const uint32_t before = (uint32_t)__popcll(__ballot(k && P < g0));
            const uint64_t M = __ballot(mark[lane] == (uint8_t)tag);
            const uint32_t g = g0 + (uint32_t)lane;
            it.valid = g < K;
            const uint32_t rk = before + (uint32_t)__popcll(M & ((2ull << lane) - 1ull)) - 1u;
            it.src = it.valid ? (dense ? (int)(rk & 63u) : (int)list[rk & 63u]) : 0;
            const uint32_t Eghi = onehi ? Ehi0 : (uint32_t)__shfl((int)Ehi, it.src);
            const uint64_t Eg = ((uint64_t)Eghi << 32) | (uint32_t)__shfl((int)Elo, it.src);
            // one shuffle for both: a frame that holds chunks is at most 1536 B, a prefix at most 1024
            // (two shuffles measured the same: IMIX 5036 vs 5041 GB/s, one process)
            const uint32_t PLg = (uint32_t)__shfl((int)PL, it.src);
            const uint32_t Lg = PLg >> 16, Pg = PLg & 0xFFFFu;
            it.c = it.valid ? g - Pg : 0u;   // chunk index back from the frame end
            it.cstart = (int64_t)Eg - (int64_t)kChunkBytes * (int64_t)(it.c + 1);
            // bytes of the window before the frame start: (Eg - Lg) - cstart
            it.zr = it.valid ? clamp_zr((int64_t)kChunkBytes * (int64_t)(it.c + 1) - (int64_t)Lg) : kChunkBytes;
        };
        auto issue = [&](FlatItem &it) { issue_any<TINY>(p, it.cstart, it.valid && it.zr < kChunkBytes, it.ch); };
        auto prep = [&](uint32_t g0, uint32_t tag, FlatItem &it) {
            deal(g0, tag, it);
            issue(it);
        };
        auto finish = [&](const FlatItem &it) {
#ifdef FCS_FLAT_NOCRC   // measurement-only build: loads and dealing without the CRC work (wrong FCS)
            uint32_t v = it.ch.x6 ^ it.c;
#pragma unroll
            for (int q = 0; q < 6; q++) v ^= it.ch.x[q].x ^ it.ch.x[q].y ^ it.ch.x[q].z ^ it.ch.x[q].w;
#else
            // lanes past the window's chunks and the dummy chunk of an empty frame (zr = 96) are discarded
            const uint32_t own = chunk_value<TINY>(lds, it.ch, it.zr, it.zr < kChunkBytes ? it.zr : 0,
                                                   it.valid ? inv_start(lds, it.zr) : 0u, base0, base1);
            const uint32_t v = chunk_shift(lds, own, it.c & 15u);
#endif
            if (it.valid && v) atomicXor(&acc[it.src], v);
        };
#ifdef FCS_FLAT_PIPE   // measurement-only build: the next item's loads in flight during this one
        if (K) {
            FlatItem A, B;
            prep(0, 1, A);
            uint32_t g0 = 64, tag = 2;
            while (true) {
                if (g0 >= K) { finish(A); break; }
                prep(g0, tag, B);
                finish(A);
                g0 += 64; tag++;
                if (g0 >= K) { finish(B); break; }
                prep(g0, tag, A);
                finish(B);
                g0 += 64; tag++;
            }
        }
#elif defined(FCS_FLAT_DEAL_AHEAD)   // measurement-only: the next item dealt while this item's loads fly
        if (K) {
            FlatItem it, nx;
            deal(0, 1, it);
            for (uint32_t g0 = 0, tag = 1; g0 < K; g0 += 64, tag++) {
                issue(it);
                const bool more = g0 + 64 < K;
                if (more) deal(g0 + 64, tag + 1, nx);
                finish(it);
                if (more) {
                    it.src = nx.src;
                    it.zr = nx.zr;
                    it.c = nx.c;
                    it.valid = nx.valid;
                    it.cstart = nx.cstart;
                }
            }
        }
#else
        for (uint32_t g0 = 0, tag = 1; g0 < K; g0 += 64, tag++) {
            FlatItem it;
            prep(g0, tag, it);
            finish(it);
        }
#endif

        // ---- frames over 1536 B: 16 lanes each, 4 per item, segment by segment ----
        const uint64_t xmask = __ballot(multi);
        const uint32_t nx = (uint32_t)__popcll(xmask);
        if (nx) {
            const uint32_t rx = __builtin_amdgcn_mbcnt_hi((uint32_t)(xmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)xmask, 0u));
            if (multi) mark[rx] = (uint8_t)lane;   // the marks are free again: reuse them as the multi list
            wave_lds_sync();
            for (uint32_t t = 0; t < nx; t += 4) {
                const uint32_t rnk = t + (uint32_t)(lane >> 4);
                const bool valid = rnk < nx;
                const int src = valid ? (int)mark[rnk] : 0;
                const uint64_t Eq = ((uint64_t)(uint32_t)__shfl((int)Ehi, src) << 32) | (uint32_t)__shfl((int)Elo, src);
                const uint32_t Lq = (uint32_t)__shfl((int)L, src);
                const uint32_t m = valid ? (Lq + (kSegBytes - 1)) / kSegBytes : 0u;
                uint32_t s = 0;
                for (uint32_t q = 0; __any(q < m); q++) {
                    const bool on = q < m;
                    const int64_t cstart = (int64_t)Eq - (int64_t)kSegBytes * (int64_t)(m - 1 - q) -
                                           (int64_t)kChunkBytes * (j + 1);
                    const int zr = (on && q == 0) ? clamp_zr((int64_t)(Eq - Lq) - cstart) : (on ? -1 : kChunkBytes);
                    Chunk cc;
                    issue_any<TINY>(p, cstart, on && zr < kChunkBytes, cc);
                    const uint32_t r = chunk_value<TINY>(lds, cc, zr, on ? zr : 0, (on && q == 0) ? inv_start(lds, zr) : 0u,
                                                         base0, base1);
                    s = on ? (q == 0 ? r : uniform_shift<kLdsJump>(lds, s, r)) : s;
                }
                const uint32_t v = row_xor(chunk_shift(lds, s, (uint32_t)j));
                if (valid && j == 15) acc[src] = v;
            }
            if (multi) mark[rx] = 0;
        }

        // ---- one coalesced store per window; clear the window state ----
        wave_lds_sync();
        const uint32_t a = acc[lane];
        emit(p, lds, act, f, L ? ~a : 0u);
        acc[lane] = 0u;
        mark[lane] = 0;
    }
    flush_bad(p, lds);
}

// ---------------------------------------------------------------------------------------------
// Shared by the LDS-DMA variable-length kernels (fcs_span_kernel, and the measurement-only
// fcs_flatdma_kernel): the 32 KiB slice tables of fcs_dma_kernel and, in the row holes, the
// c-indexed shift tables A_{96c} (nibble t of table c at hole 4c + t/2, +64 B for odd t), the A_48
// merge table and INV of fcs_dma_kernel, A_1536 for frames over 1536 B, and each wave's window
// scratch (accumulators, marks, frame lists).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kFdJumpHole = 152;                  // A_1536: 4 holes
constexpr uint32_t kFdWaveHole = 160;                  // 4 holes per wave: acc[0..31], acc[32..63], marks | list, multi list
static_assert(kDmaInvHole + 4 <= kFdJumpHole && kFdWaveHole + 4 * 16 <= 256, "holes");

__device__ __forceinline__ uint32_t fd_acc_addr(uint32_t wave, uint32_t i) {
    return dma_hole(kFdWaveHole + 4u * wave + (i >> 5)) + (i & 31u) * 4u;
}

// A_{96c}(s), c = 0..15, from the c-indexed hole tables.
__device__ __forceinline__ uint32_t fd_chunk_shift(const uint8_t *lds, uint32_t s, uint32_t c) {
    uint32_t r[8];
    const uint32_t base = dma_hole(4u * c);
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        r[t] = lds_rd(lds, base + (sh & 0x3Cu) + 256u * (uint32_t)(t >> 1) + 64u * (uint32_t)(t & 1));
    }
    return xor9(r, 0u);
}

// A_1536(s) ^ extra from its hole table.
__device__ __forceinline__ uint32_t fd_jump(const uint8_t *lds, uint32_t s, uint32_t extra) {
    uint32_t r[8];
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        r[t] = lds_rd(lds, dma_hole(kFdJumpHole + (uint32_t)(t >> 1)) + 64u * (uint32_t)(t & 1) + (sh & 0x3Cu));
    }
    return xor9(r, extra);
}

__device__ __forceinline__ uint32_t fd_inv(const uint8_t *lds, int zr) {
    const int zi = zr < 0 ? 0 : (zr > kChunkBytes - 1 ? kChunkBytes - 1 : zr);
    const uint32_t iv = lds_rd(lds, dma_hole(kDmaInvHole + (uint32_t)zi / 32u) + (uint32_t)(zi % 32) * 4u);
    return (zr >= 0 && zr < kChunkBytes) ? iv : 0u;
}

// The words of a register-loaded chunk, realigned to its start (arena edge undone).
__device__ __forceinline__ void fd_chunk_words(const Chunk &c, uint32_t (&w)[kChunkWords]) {
    uint32_t d[kChunkWords + 1];
#pragma unroll
    for (int q = 0; q < 6; q++) {
        d[4 * q] = c.x[q].x;
        d[4 * q + 1] = c.x[q].y;
        d[4 * q + 2] = c.x[q].z;
        d[4 * q + 3] = c.x[q].w;
    }
    d[kChunkWords] = c.x6;
    if (__any(c.dlead)) shift_up(d, c.dlead);
#pragma unroll
    for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], c.r);
}

// A chunk's register before its shift: bytes before the frame start masked (groups of 4 words up
// to the wave's largest claim zb, as chunk_value), x0 injected, two 12-word chains on the 32 KiB
// tables, A_48 merge.
__device__ __forceinline__ uint32_t fd_value(const uint8_t *lds, uint32_t (&w)[kChunkWords], int zr, int zb, uint32_t x0,
                                             const uint32_t (&B)[4], const uint32_t (&SEL)[4]) {
    const int zr8 = 8 * zr;
#pragma unroll
    for (int g = 0; g < kChunkWords / 4; g++) {
        if (!__any(zb > 16 * g)) break;
#pragma unroll
        for (int i = 4 * g; i < 4 * g + 4; i++) {
            w[i] = clear_low_bits(w[i], zr8 - 32 * i);
        }
    }
    uint32_t xa = x0 ^ w[0], xb = w[12];
#pragma unroll
    for (int i = 0; i < 12; i++) {
        xa = step4_l8(lds, xa, i < 11 ? w[i + 1] : 0u, B, SEL);
        xb = step4_l8(lds, xb, i < 11 ? w[13 + i] : 0u, B, SEL);
    }
    return merge_shift_dma(lds, 0, xa, xb);
}

// Table image of the variable-length LDS-DMA kernels (layout above); zeroes every wave's scratch.
template <int NT = kWgThreads>
__device__ __forceinline__ void stage_fd_tables(const KParams &p, uint8_t *lds, int tid) {
    for (int i = tid; i < 2048; i += NT) {   // slice tables as fcs_dma_kernel
        const uint32_t v = p.blob[kBlobSlice + 256 * (3 - ((i & 7) >> 1)) + (i >> 3)];
        u32x4 vv = {v, v, v, v};
        *reinterpret_cast<u32x4 *>(lds + (uint32_t)(i >> 3) * 256u + (uint32_t)(i & 7) * 16u) = vv;
    }
    for (int i = tid; i < 16 * 128; i += NT) {   // A_{96c}: table c, nibble t, entry e
        const int c = i >> 7, t = (i >> 4) & 7, e = i & 15;
        *reinterpret_cast<uint32_t *>(lds + dma_hole(4u * (uint32_t)c + (uint32_t)(t >> 1)) + 64u * (uint32_t)(t & 1) +
                                      4u * (uint32_t)e) = p.blob[kBlobFlat + c * (kFlatStride / 4) + t * 16 + e];
    }
    for (int i = tid; i < 128; i += NT) {   // A_48 (merge table 0 of fcs_dma_kernel) and A_1536
        const int t = (i >> 4) & 7, e = i & 15;
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kDmaMergeHole + (uint32_t)(t >> 1)) + 64u * (uint32_t)(t & 1) +
                                      4u * (uint32_t)e) = p.blob[kBlobMerge + (kDmaChainWords / 2 - 1) * 128 + i];
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kFdJumpHole + (uint32_t)(t >> 1)) + 64u * (uint32_t)(t & 1) +
                                      4u * (uint32_t)e) = p.blob[kBlobJump + i];
    }
    for (int i = tid; i < kChunkBytes; i += NT)
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kDmaInvHole + (uint32_t)i / 32u) + (uint32_t)(i % 32) * 4u) =
            p.blob[kBlobInv + i];
    for (int i = tid; i < 16 * 4 * 32; i += NT)   // window scratch of every wave: zero
        *reinterpret_cast<uint32_t *>(lds + dma_hole(kFdWaveHole + (uint32_t)i / 32u) + (uint32_t)(i % 32) * 4u) = 0u;
}

#ifdef FCS_FLAT2
// ---------------------------------------------------------------------------------------------
// MEASUREMENT-ONLY (-DFCS_FLAT2; rejected, DESIGN.md §3.3: 2 x 8 waves IMIX +2 %, 576 B -2 %;
// 2 x 10 and 2 x 12 waves slower or mixed).
// The flat chunk stream at two workgroups per CU (fcs_flat2_kernel). fcs_flat_kernel runs slower
// with fewer waves per CU (IMIX, one process: 12 waves 4828, 14 waves 5078, 16 waves 5286 GB/s),
// and 16 is one workgroup's limit. This form
// keeps the flat kernel's dealing and chunk work but takes the compact 64 KiB table image of the
// LDS-DMA kernels (32 KiB of 8-replica slice tables; A_{96c}, A_48, A_1536, INV and each wave's
// accumulators, marks and lists in the row holes: stage_fd_tables), so two workgroups of
// kFlat2Threads fit one CU's LDS, and its registers are held to kFlat2Waves / 4 waves per SIMD.
// ---------------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT, 2) void fcs_flat2_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDmaRing];
    static_assert(NT / 64 <= 16, "wave scratch holds 16 waves");
    const int tid = threadIdx.x;
    stage_fd_tables<NT>(p, lds, tid);
    init_bad<kDmaBad>(lds);
    __syncthreads();

    const int lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & (kGroup - 1);
    const uint32_t h = (uint32_t)(lane >> 3) & 3u, r4 = (uint32_t)(lane & 7) * 4u;
    const uint32_t B[4] = {r4 + 32u * (0u ^ h), r4 + 32u * (1u ^ h), r4 + 32u * (2u ^ h), r4 + 32u * (3u ^ h)};
    const uint32_t SEL[4] = {0x0C0C0400u + ((0u ^ h) << 8), 0x0C0C0400u + ((1u ^ h) << 8),
                             0x0C0C0400u + ((2u ^ h) << 8), 0x0C0C0400u + ((3u ^ h) << 8)};
    uint8_t *mark = lds + dma_hole(kFdWaveHole + 4u * wave + 2u);
    uint8_t *list = mark + 64;
    uint8_t *mlist = lds + dma_hole(kFdWaveHole + 4u * wave + 3u);
    auto acc = [&](uint32_t i) { return reinterpret_cast<uint32_t *>(lds + fd_acc_addr(wave, i)); };

    Dispenser D(p.ctr, (p.n + 63) >> 6, (uint64_t)gridDim.x * (NT / 64),
                (uint64_t)blockIdx.x * (NT / 64) + (uint64_t)wave, lane, 100, 1, FCS_FLAT_CHUNK_MAX);
    for (uint64_t win = D.first(); win != Dispenser::kEnd; win = D.next(win)) {
        const uint64_t w0 = win * 64;
        // ---- window metadata: lane i <-> frame w0 + i ----
        const uint64_t f = w0 + lane;
        const bool act = f < p.n;
        const uint32_t L = act ? (p.len ? p.len[f] : p.flen) : 0u;   // len == null: fixed length
        const uint64_t E = act ? p.base + (p.off ? p.off[f] : f * p.stride) + L : p.lo4;
        const bool multi = act && L > (uint32_t)kSegBytes;
        const uint32_t k = (!act || multi) ? 0u : (L ? (L + kChunkBytes - 1) / kChunkBytes : 1u);
        uint32_t incl = k;   // inclusive prefix over the window
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t P = incl - k;
        const uint32_t K = (uint32_t)__shfl((int)incl, 63);
        const uint64_t fmask = __ballot(k != 0);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fmask, 0u));
        mark[lane] = 0;
        if (k) list[rank] = (uint8_t)lane;
        wave_lds_sync();
        const uint32_t Elo = (uint32_t)E, Ehi = (uint32_t)(E >> 32);
        // no frame over 1536 B: a chunk's frame rank is its frame's lane; frame ends in one 4 GiB page
        const bool dense = __ballot(multi) == 0;
        const uint32_t Ehi0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)Ehi);
        const bool onehi = __ballot(Ehi != Ehi0) == 0;

        // one item = 64 chunks: lane -> (frame, chunk), its loads, its chunk value into the frame
        for (uint32_t g0 = 0, tag = 1; g0 < K; g0 += 64, tag++) {
            if (k && P >= g0 && P < g0 + 64) mark[P - g0] = (uint8_t)tag;
            wave_lds_sync();
            const uint32_t before = (uint32_t)__popcll(__ballot(k && P < g0));
            const uint64_t M = __ballot(mark[lane] == (uint8_t)tag);
            const uint32_t g = g0 + (uint32_t)lane;
            const bool valid = g < K;
            const uint32_t rk = before + (uint32_t)__popcll(M & ((2ull << lane) - 1ull)) - 1u;
            const int src = valid ? (dense ? (int)(rk & 63u) : (int)list[rk & 63u]) : 0;
            const uint32_t Eghi = onehi ? Ehi0 : (uint32_t)__shfl((int)Ehi, src);
            const uint64_t Eg = ((uint64_t)Eghi << 32) | (uint32_t)__shfl((int)Elo, src);
            const uint32_t Lg = (uint32_t)__shfl((int)L, src);
            const uint32_t Pg = (uint32_t)__shfl((int)P, src);
            const uint32_t c = valid ? g - Pg : 0u;   // chunk index back from the frame end
            const int64_t cstart = (int64_t)Eg - (int64_t)kChunkBytes * (int64_t)(c + 1);
            const int zr = valid ? clamp_zr((int64_t)(Eg - Lg) - cstart) : kChunkBytes;
            Chunk ch;
            issue_any<false>(p, cstart, valid && zr < kChunkBytes, ch);
            uint32_t w[kChunkWords];
            fd_chunk_words(ch, w);
            // lanes past the window's chunks and the dummy chunk of an empty frame (zr = 96) are discarded
            const uint32_t own = fd_value(lds, w, zr, zr < kChunkBytes ? zr : 0, valid ? fd_inv(lds, zr) : 0u, B, SEL);
            const uint32_t v = fd_chunk_shift(lds, own, c & 15u);
            if (valid && v) atomicXor(acc((uint32_t)src), v);
        }

        // ---- frames over 1536 B: 16 lanes each, 4 per item, segment by segment ----
        const uint64_t xmask = __ballot(multi);
        const uint32_t nx = (uint32_t)__popcll(xmask);
        if (nx) {
            const uint32_t rx = __builtin_amdgcn_mbcnt_hi((uint32_t)(xmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)xmask, 0u));
            if (multi) mlist[rx] = (uint8_t)lane;
            wave_lds_sync();
            for (uint32_t t = 0; t < nx; t += 4) {
                const uint32_t rnk = t + (uint32_t)(lane >> 4);
                const bool valid = rnk < nx;
                const int src = valid ? (int)mlist[rnk] : 0;
                const uint64_t Eq = ((uint64_t)(uint32_t)__shfl((int)Ehi, src) << 32) | (uint32_t)__shfl((int)Elo, src);
                const uint32_t Lq = (uint32_t)__shfl((int)L, src);
                const uint32_t m = valid ? (Lq + (kSegBytes - 1)) / kSegBytes : 0u;
                uint32_t s = 0;
                for (uint32_t q = 0; __any(q < m); q++) {
                    const bool on = q < m;
                    const int64_t cstart = (int64_t)Eq - (int64_t)kSegBytes * (int64_t)(m - 1 - q) -
                                           (int64_t)kChunkBytes * (j + 1);
                    const int zr = (on && q == 0) ? clamp_zr((int64_t)(Eq - Lq) - cstart) : (on ? -1 : kChunkBytes);
                    Chunk cc;
                    issue_any<false>(p, cstart, on && zr < kChunkBytes, cc);
                    uint32_t w[kChunkWords];
                    fd_chunk_words(cc, w);
                    const uint32_t r = fd_value(lds, w, zr, on ? zr : 0, (on && q == 0) ? fd_inv(lds, zr) : 0u, B, SEL);
                    s = on ? (q == 0 ? r : fd_jump(lds, s, r)) : s;
                }
                const uint32_t v = row_xor(fd_chunk_shift(lds, s, (uint32_t)j));
                if (valid && j == 15) *acc((uint32_t)src) = v;
            }
        }

        // ---- one coalesced store per window; clear the accumulators ----
        wave_lds_sync();
        const uint32_t a = *acc((uint32_t)lane);
        emit<kDmaBad>(p, lds, act, f, L ? ~a : 0u);
        *acc((uint32_t)lane) = 0u;
    }
    flush_bad<kDmaBad>(p, lds);
}
#endif  // FCS_FLAT2

#ifdef FCS_FLATDMA
constexpr uint32_t kFdSlotBytes = 6144;                // 64 lanes x 96 B, piece i of lane l at 1024 i + 16 l
// ---------------------------------------------------------------------------------------------
// MEASUREMENT-ONLY (-DFCS_FLATDMA; rejected: IMIX 4629 vs 5200 GB/s).
// Variable-length frames, flat chunk stream, chunk windows staged through LDS by DMA
// (fcs_flatdma_kernel; replaces fcs_flat_kernel<false> in -DFCS_FLATDMA builds).
// The dealing of fcs_flat_kernel (64-frame windows, 64 chunks per item, frame-start marks), but
// each lane copies its own 96-byte window into the wave's LDS slot with six
// global_load_lds_dwordx4 at the window's exact byte address: gfx950's LDS-DMA honours any byte
// alignment (tools/microbench/glds_align.hip), so no realignment is needed and no VGPR holds the
// bytes in flight. Lane l's 16-byte piece i lands at slot + 1024 i + 16 l and comes back with one
// ds_read_b128 per piece (16 lanes per 256-B bank row: 4 cycles, the minimum; random 16-B pieces
// would cost 12, tools/microbench/lds_pat.hip). A wave deals its next item and issues that item's
// DMA as soon as the current item's words are in registers, so the next item's bytes land while
// the current item's CRC work runs (fcs_flat_kernel waits for each item's loads with nothing else
// to do). An item whose windows reach before the arena start (the frames at the arena's first 96
// bytes) is loaded into registers instead, with the arena-edge shift of the other kernels.
// Tables: the 32 KiB slice tables of fcs_dma_kernel (step4_l8) and, in the row holes, the
// c-indexed shift tables A_{96c} (nibble t of table c at hole 4c + t/2, +64 B for odd t), the A_48
// merge table and INV of fcs_dma_kernel, A_1536 for frames over 1536 B, and each wave's window
// scratch (accumulators, marks, frame lists).
// ---------------------------------------------------------------------------------------------
#ifndef FCS_FD_AUX   // cache policy of the window DMA (measurement-only override)
#define FCS_FD_AUX 0
#endif

__global__ __launch_bounds__(kWgThreads, 1) void fcs_flatdma_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDmaRing + 16 * kFdSlotBytes];
    static_assert(kWgThreads / 64 <= 16, "slots");
    const int tid = threadIdx.x;
    stage_fd_tables(p, lds, tid);
    init_bad<kDmaBad>(lds);
    __syncthreads();

    const int lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & (kGroup - 1);
    const uint32_t h = (uint32_t)(lane >> 3) & 3u, r4 = (uint32_t)(lane & 7) * 4u;
    const uint32_t B[4] = {r4 + 32u * (0u ^ h), r4 + 32u * (1u ^ h), r4 + 32u * (2u ^ h), r4 + 32u * (3u ^ h)};
    const uint32_t SEL[4] = {0x0C0C0400u + ((0u ^ h) << 8), 0x0C0C0400u + ((1u ^ h) << 8),
                             0x0C0C0400u + ((2u ^ h) << 8), 0x0C0C0400u + ((3u ^ h) << 8)};
    uint8_t *slot = lds + kDmaRing + wave * kFdSlotBytes;
    uint8_t *mark = lds + dma_hole(kFdWaveHole + 4u * wave + 2u);
    uint8_t *list = mark + 64;
    uint8_t *mlist = lds + dma_hole(kFdWaveHole + 4u * wave + 3u);
    const uint32_t acc_lane = fd_acc_addr(wave, (uint32_t)lane);

    struct It {
        int src, zr;
        uint32_t c;
        int64_t cstart;
        uint64_t base;      // chunk-major DMA: lane 0's window start, and this lane's offset from it
        int relv;
        bool valid, rare;   // rare (wave-uniform): a window reaches before the arena start
    };

    Dispenser D(p.ctr, (p.n + 63) >> 6, (uint64_t)gridDim.x * (kWgThreads / 64),
                (uint64_t)blockIdx.x * (kWgThreads / 64) + (uint64_t)wave, lane, 100, 1, FCS_FLAT_CHUNK_MAX);
    uint32_t tagc = 0;   // mark tags: distinct within a window (reset with the marks)
    for (uint64_t win = D.first(); win != Dispenser::kEnd; win = D.next(win)) {
        const uint64_t w0 = win * 64;
        // ---- window metadata: lane i <-> frame w0 + i ----
        const uint64_t f = w0 + lane;
        const bool act = f < p.n;
        const uint32_t L = act ? (p.len ? p.len[f] : p.flen) : 0u;   // len == null: fixed length
        const uint64_t E = act ? p.base + (p.off ? p.off[f] : f * p.stride) + L : p.lo4;
        const bool multi = act && L > (uint32_t)kSegBytes;
        const uint32_t k = (!act || multi) ? 0u : (L ? (L + kChunkBytes - 1) / kChunkBytes : 1u);
        uint32_t incl = k;   // inclusive prefix over the window
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t P = incl - k;
        const uint32_t K = (uint32_t)__shfl((int)incl, 63);
        const uint64_t fmask = __ballot(k != 0);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fmask, 0u));
        mark[lane] = 0;
        if (k) list[rank] = (uint8_t)lane;
        wave_lds_sync();
        const uint32_t Elo = (uint32_t)E, Ehi = (uint32_t)(E >> 32);
        tagc = 0;

        // deal item g0: lane -> (frame, chunk), then issue its window DMA
        auto prep = [&](uint32_t g0, It &it) {
            const uint8_t tag = (uint8_t)++tagc;
            if (k && P >= g0 && P < g0 + 64) mark[P - g0] = tag;
            wave_lds_sync();
            const uint32_t before = (uint32_t)__popcll(__ballot(k && P < g0));
            const uint64_t M = __ballot(mark[lane] == tag);
            const uint32_t g = g0 + (uint32_t)lane;
            it.valid = g < K;
            const uint32_t rk = before + (uint32_t)__popcll(M & ((2ull << lane) - 1ull)) - 1u;
            it.src = it.valid ? (int)list[rk & 63u] : 0;
            const uint64_t Eg = ((uint64_t)(uint32_t)__shfl((int)Ehi, it.src) << 32) | (uint32_t)__shfl((int)Elo, it.src);
            const uint32_t Lg = (uint32_t)__shfl((int)L, it.src);
            const uint32_t Pg = (uint32_t)__shfl((int)P, it.src);
            it.c = it.valid ? g - Pg : 0u;   // chunk index back from the frame end
            it.cstart = (int64_t)Eg - (int64_t)kChunkBytes * (int64_t)(it.c + 1);
            it.zr = it.valid ? clamp_zr((int64_t)(Eg - Lg) - it.cstart) : kChunkBytes;
            const bool need = it.valid && it.zr < kChunkBytes;
            // chunk-major DMA: instruction i, lane l copies piece m of chunk q (6 q + m = 64 i + l)
            // to slot + 96 q + 16 m, so the 6 lanes of a chunk read its 96 contiguous bytes and
            // consecutive chunks of a frame are adjacent runs; chunk addresses travel as 32-bit
            // offsets from lane 0's window
            const uint64_t base = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)((uint64_t)it.cstart >> 32)) << 32) |
                                  (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)it.cstart);
            const int64_t rel = it.cstart - (int64_t)base;
            const bool far = rel < -(int64_t)0x3FFFFFFF || rel > (int64_t)0x3FFFFFFF;
            it.rare = __any(need && (it.cstart < (int64_t)p.lo4 || far));
            it.base = base;
            it.relv = need ? (int)rel : (int)0x80000000;
        };
        // the item's window DMA (after its dealing, once the slot is free)
        auto dma = [&](const It &it) {
            if (!it.rare) {
                typedef __attribute__((address_space(3))) void lds_void;
#pragma unroll
                for (int i = 0; i < 6; i++) {
                    const uint32_t t = 64u * (uint32_t)i + (uint32_t)lane, q = t / 6u, m = t - 6u * q;
                    const int rq = __shfl(it.relv, (int)q);
                    if (rq != (int)0x80000000)
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(it.base + (int64_t)rq + 16 * m),
                                                         (lds_void *)(slot + 1024 * i), 16, 0, FCS_FD_AUX);
                }
            }
        };
        auto finish = [&](const It &it, uint32_t (&w)[kChunkWords]) {
            // lanes past the window's chunks and the dummy chunk of an empty frame (zr = 96) are discarded
            const uint32_t own = fd_value(lds, w, it.zr, it.zr < kChunkBytes ? it.zr : 0, it.valid ? fd_inv(lds, it.zr) : 0u,
                                          B, SEL);
            const uint32_t v = fd_chunk_shift(lds, own, it.c & 15u);
            if (it.valid && v) atomicXor(reinterpret_cast<uint32_t *>(lds + fd_acc_addr(wave, (uint32_t)it.src)), v);
        };

        if (K) {
            It cur;
            prep(0, cur);
            dma(cur);
            for (uint32_t g0 = 0; g0 < K; g0 += 64) {
                uint32_t w[kChunkWords];
                // the next item's dealing first: its LDS round trips overlap this item's DMA wait
                It nxt;
                nxt.valid = false;
                const bool more = g0 + 64 < K;
                if (more) prep(g0 + 64, nxt);
                if (!cur.rare) {
                    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this item's window DMA has landed
#pragma unroll
                    for (int i = 0; i < 6; i++) {
                        const u32x4 x = *reinterpret_cast<const u32x4 *>(slot + 96 * lane + 16 * i);
                        w[4 * i] = x.x;
                        w[4 * i + 1] = x.y;
                        w[4 * i + 2] = x.z;
                        w[4 * i + 3] = x.w;
                    }
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next DMA
                } else {   // the arena start: register loads with the edge shift
                    Chunk ch;
                    issue_any<false>(p, cur.cstart, cur.valid && cur.zr < kChunkBytes, ch);
                    fd_chunk_words(ch, w);
                }
                if (more) dma(nxt);
                finish(cur, w);
                cur = nxt;
            }
        }

        // ---- frames over 1536 B: 16 lanes each, 4 per item, segment by segment (register loads) ----
        const uint64_t xmask = __ballot(multi);
        const uint32_t nx = (uint32_t)__popcll(xmask);
        if (nx) {
            const uint32_t rx = __builtin_amdgcn_mbcnt_hi((uint32_t)(xmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)xmask, 0u));
            if (multi) mlist[rx] = (uint8_t)lane;
            wave_lds_sync();
            for (uint32_t t = 0; t < nx; t += 4) {
                const uint32_t rnk = t + (uint32_t)(lane >> 4);
                const bool valid = rnk < nx;
                const int src = valid ? (int)mlist[rnk] : 0;
                const uint64_t Eq = ((uint64_t)(uint32_t)__shfl((int)Ehi, src) << 32) | (uint32_t)__shfl((int)Elo, src);
                const uint32_t Lq = (uint32_t)__shfl((int)L, src);
                const uint32_t m = valid ? (Lq + (kSegBytes - 1)) / kSegBytes : 0u;
                uint32_t s = 0;
                for (uint32_t q = 0; __any(q < m); q++) {
                    const bool on = q < m;
                    const int64_t cstart = (int64_t)Eq - (int64_t)kSegBytes * (int64_t)(m - 1 - q) -
                                           (int64_t)kChunkBytes * (j + 1);
                    const int zr = (on && q == 0) ? clamp_zr((int64_t)(Eq - Lq) - cstart) : (on ? -1 : kChunkBytes);
                    Chunk cc;
                    issue_any<false>(p, cstart, on && zr < kChunkBytes, cc);
                    uint32_t w[kChunkWords];
                    fd_chunk_words(cc, w);
                    const uint32_t r = fd_value(lds, w, zr, on ? zr : 0, (on && q == 0) ? fd_inv(lds, zr) : 0u, B, SEL);
                    s = on ? (q == 0 ? r : fd_jump(lds, s, r)) : s;
                }
                const uint32_t v = row_xor(fd_chunk_shift(lds, s, (uint32_t)j));
                if (valid && j == 15) *reinterpret_cast<uint32_t *>(lds + fd_acc_addr(wave, (uint32_t)src)) = v;
            }
        }

        // ---- one coalesced store per window; clear the accumulators ----
        wave_lds_sync();
        uint32_t *accp = reinterpret_cast<uint32_t *>(lds + acc_lane);
        const uint32_t a = *accp;
        emit<kDmaBad>(p, lds, act, f, L ? ~a : 0u);
        *accp = 0u;
    }
    flush_bad<kDmaBad>(p, lds);
}
#endif  // FCS_FLATDMA

#ifdef FCS_SPAN
// ---------------------------------------------------------------------------------------------
// MEASUREMENT-ONLY (-DFCS_SPAN; rejected: IMIX 4408 vs 4977 GB/s for fcs_flat_kernel in one
// process). Its loads alone run at 5734-6130 GB/s against the flat kernel's 5344,
// but its CRC work is not hidden behind them: per item it adds the LDS-DMA writes, seven 16-B
// window reads and a 16-B realignment to the chain's table lookups, and the CU's VALU and LDS
// pipes then limit it.
// Variable-length frames, flat chunk stream staged through LDS by span DMA (fcs_span_kernel;
// replaces fcs_flat_kernel<false> for windowed batches in -DFCS_SPAN builds).
// The dealing of fcs_flat_kernel (64-frame windows, 64 chunks per item, frame-start marks), with a
// frame's chunks dealt front to back: window chunk g is chunk k - 1 - (g - P) back from its frame's
// end (k chunks, P the frame's first chunk). An item's 64 chunks then lie in arena order, and for
// packed frames inside one span of at most 64 x 96 bytes (frame-aligned chunks overlap at frame
// fronts, they never leave gaps). That span is one LDS-DMA of up to six 1 KiB rows into the wave's
// 6 KiB slot: the coalesced rows of fcs_dma_kernel instead of 64 scattered 96-B windows. Its start
// and end are wave-uniform scalar work (the frames holding the item's first and last chunk: a
// ballot over the prefix, readlanes), independent of the per-lane dealing, so the next item's DMA
// is issued as soon as the current item's windows are in registers; the current item's CRC work
// and the next item's dealing (marks, ballots, bpermutes) run while it flies. A lane reads its
// 96-B window at its byte offset in the slot (25 dwords, realigned as in fcs_dma_kernel).
// An item whose windows do not all lie in its slot (gaps between frames, offsets out of order, a
// frame over 1536 B between two others) loads them into registers instead (issue_any, the
// arena-edge path of the other kernels). Frames over 1536 B take the segment loop of
// fcs_flat_kernel. The next window's offsets and lengths are loaded at the start of the current one.
// ---------------------------------------------------------------------------------------------
struct SpanDma {
    uint64_t src;    // 16-B aligned address of the slot's first byte
    uint32_t need;   // slot bytes up to the end of the item's last chunk
    bool rare;       // wave-uniform: the item's chunks do not fit the slot (register loads, no DMA)
};

// The item's span: 1 KiB rows as far as its bytes reach. The first and the last row keep the
// default cache policy (their 128-B lines are shared with the neighbouring items), the rows
// between are non-temporal, as in dma_item.
__device__ __forceinline__ void span_dma(const uint8_t *slot, const SpanDma &sd, int lane) {
    typedef __attribute__((address_space(3))) void lds_void;
    const uint64_t a = sd.src + 16 * (uint64_t)lane, b = a + 4096;
    lds_void *la = (lds_void *)slot, *lb = (lds_void *)(slot + 4096);
    const uint32_t o = 16u * (uint32_t)lane, need = sd.need;
    const uint32_t last = (need - 1u) >> 10;   // wave-uniform
    if (o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 0, FCS_DMA_EDGE_AUX);
    if (1024u + o < need) {
        if (last == 1) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 1024, FCS_DMA_EDGE_AUX);
        else __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 1024, FCS_DMA_AUX);
    }
    if (2048u + o < need) {
        if (last == 2) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 2048, FCS_DMA_EDGE_AUX);
        else __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 2048, FCS_DMA_AUX);
    }
    if (3072u + o < need) {
        if (last == 3) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 3072, FCS_DMA_EDGE_AUX);
        else __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 3072, FCS_DMA_AUX);
    }
    if (4096u + o < need) {
        if (last == 4) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(b), lb, 16, 0, FCS_DMA_EDGE_AUX);
        else __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(b), lb, 16, 0, FCS_DMA_AUX);
    }
    if (5120u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(b), lb, 16, 1024, FCS_DMA_EDGE_AUX);
}

__global__ __launch_bounds__(kWgThreads, 1) void fcs_span_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDmaRing + 16 * kDmaItemBytes];
    static_assert(kWgThreads / 64 <= 16, "slots");
    const int tid = threadIdx.x;
    stage_fd_tables(p, lds, tid);
    init_bad<kDmaBad>(lds);
    __syncthreads();

    const int lane = tid & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & (kGroup - 1);
    const uint32_t h = (uint32_t)(lane >> 3) & 3u, r4 = (uint32_t)(lane & 7) * 4u;
    const uint32_t B[4] = {r4 + 32u * (0u ^ h), r4 + 32u * (1u ^ h), r4 + 32u * (2u ^ h), r4 + 32u * (3u ^ h)};
    const uint32_t SEL[4] = {0x0C0C0400u + ((0u ^ h) << 8), 0x0C0C0400u + ((1u ^ h) << 8),
                             0x0C0C0400u + ((2u ^ h) << 8), 0x0C0C0400u + ((3u ^ h) << 8)};
    const uint8_t *slot = lds + kDmaRing + wave * kDmaItemBytes;
    uint8_t *mark = lds + dma_hole(kFdWaveHole + 4u * wave + 2u);
    uint8_t *list = mark + 64;
    uint8_t *mlist = lds + dma_hole(kFdWaveHole + 4u * wave + 3u);
    const uint32_t acc_lane = fd_acc_addr(wave, (uint32_t)lane);
    const uint64_t lo16 = p.lo4 & ~15ull;
    const uint64_t smax = ((p.hi4 + 15) & ~15ull) - kDmaItemBytes;   // last slot start (host: arena >= 2 slots)

    struct It {
        int src, zr;
        uint32_t c;
        int64_t cstart;
        bool valid, rare;
    };

    Dispenser D(p.ctr, (p.n + 63) >> 6, (uint64_t)gridDim.x * (kWgThreads / 64),
                (uint64_t)blockIdx.x * (kWgThreads / 64) + (uint64_t)wave, lane, 100, 1, FCS_FLAT_CHUNK_MAX);
    // window metadata, loaded one window ahead (raw: the loads stay in flight): lane i <-> frame 64 win + i
    auto load_meta = [&](uint64_t win, uint32_t &Lr, uint64_t &Or) {
        const uint64_t f = win * 64 + (uint64_t)lane;
        const bool act = win != Dispenser::kEnd && f < p.n;
        Lr = act ? (p.len ? p.len[f] : p.flen) : 0u;   // len == null: fixed length
        Or = act ? (p.off ? p.off[f] : f * p.stride) : 0u;
    };
    uint64_t win = D.first();
    uint32_t Ln;
    uint64_t On;
    load_meta(win, Ln, On);
    uint32_t tagc = 0;   // mark tags: distinct within a window (reset with the marks)
    while (win != Dispenser::kEnd) {
        const uint64_t w0 = win * 64;
        const uint64_t f = w0 + lane;
        const bool act = f < p.n;
        const uint32_t L = Ln;
        const uint64_t E = act ? p.base + On + L : p.lo4;
        const uint64_t nwin = D.next(win);
        load_meta(nwin, Ln, On);
        const bool multi = act && L > (uint32_t)kSegBytes;
        const uint32_t k = (!act || multi) ? 0u : (L ? (L + kChunkBytes - 1) / kChunkBytes : 1u);
        uint32_t incl = k;   // inclusive prefix over the window
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t P = incl - k;
        const uint32_t K = (uint32_t)__shfl((int)incl, 63);
        const uint64_t fmask = __ballot(k != 0);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(fmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fmask, 0u));
        mark[lane] = 0;
        if (k) list[rank] = (uint8_t)lane;
        wave_lds_sync();
        const uint32_t Elo = (uint32_t)E, Ehi = (uint32_t)(E >> 32);
        // no frame over 1536 B: the frames with chunks are lanes 0, 1, ..., so a rank is a lane
        const bool dense = __ballot(multi) == 0;
        tagc = 0;

        // wave-uniform: start address of window chunk g < K
        auto chunk_at = [&](uint32_t g) -> int64_t {
            const uint32_t rk = (uint32_t)__popcll(__ballot(k != 0 && P <= g)) - 1u;
            const int fl = dense ? (int)rk : __builtin_amdgcn_readfirstlane((int)list[rk & 63u]);
            const uint64_t Ef = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)Ehi, fl) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)Elo, fl);
            const uint32_t Lf = (uint32_t)__builtin_amdgcn_readlane((int)L, fl);
            const uint32_t Pf = (uint32_t)__builtin_amdgcn_readlane((int)P, fl);
            const uint32_t kf = Lf ? (Lf + kChunkBytes - 1) / kChunkBytes : 1u;
            return (int64_t)Ef - (int64_t)kChunkBytes * (int64_t)(kf - (g - Pf));
        };
        // the slot of item g0: from its first chunk's 16-B line to its last chunk's end
        auto span = [&](uint32_t g0) -> SpanDma {
            const uint32_t g1 = (g0 + 64 < K ? g0 + 64 : K) - 1u;
            const int64_t s0 = chunk_at(g0), e1 = chunk_at(g1) + kChunkBytes;
            SpanDma sd;
            const uint64_t a = (uint64_t)s0 & ~15ull;
            sd.src = a < lo16 ? lo16 : (a > smax ? smax : a);
            const int64_t need = e1 - (int64_t)sd.src;
            sd.rare = need <= 0 || need > (int64_t)kDmaItemBytes;
            sd.need = (uint32_t)__builtin_amdgcn_readfirstlane((int)(sd.rare ? 1u : (uint32_t)need));
            sd.src = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(sd.src >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sd.src);
            return sd;
        };
        // deal item g0: lane -> (frame, chunk); the item stays on the DMA path only if every lane's
        // frame bytes lie in the slot
        auto prep = [&](uint32_t g0, const SpanDma &sd, It &it) {
            const uint8_t tag = (uint8_t)++tagc;
            if (k && P >= g0 && P < g0 + 64) mark[P - g0] = tag;
            wave_lds_sync();
            const uint32_t before = (uint32_t)__popcll(__ballot(k && P < g0));
            const uint64_t M = __ballot(mark[lane] == tag);
            const uint32_t g = g0 + (uint32_t)lane;
            it.valid = g < K;
            const uint32_t rk = before + (uint32_t)__popcll(M & ((2ull << lane) - 1ull)) - 1u;
            it.src = it.valid ? (dense ? (int)(rk & 63u) : (int)list[rk & 63u]) : 0;
            const uint64_t Eg = ((uint64_t)(uint32_t)__shfl((int)Ehi, it.src) << 32) | (uint32_t)__shfl((int)Elo, it.src);
            const uint32_t Lg = (uint32_t)__shfl((int)L, it.src);
            const uint32_t Pg = (uint32_t)__shfl((int)P, it.src);
            const uint32_t kg = Lg ? (Lg + kChunkBytes - 1) / kChunkBytes : 1u;
            it.c = it.valid ? kg - 1u - (g - Pg) : 0u;   // chunk index back from the frame end
            it.cstart = (int64_t)Eg - (int64_t)kChunkBytes * (int64_t)(it.c + 1);
            const int64_t fs = (int64_t)(Eg - Lg);
            it.zr = it.valid ? clamp_zr(fs - it.cstart) : kChunkBytes;
            const int64_t lo = it.cstart > fs ? it.cstart : fs;
            const bool in = !it.valid || it.zr >= kChunkBytes ||
                            (lo >= (int64_t)sd.src && it.cstart + kChunkBytes <= (int64_t)sd.src + (int64_t)sd.need);
            it.rare = sd.rare || __any(!in);
        };

        if (K) {
            SpanDma sp = span(0);
            if (!sp.rare) span_dma(slot, sp, lane);
            It cur;
            prep(0, sp, cur);
            for (uint32_t g0 = 0; g0 < K; g0 += 64) {
                const bool more = g0 + 64 < K;
                SpanDma sn{0, 1u, true};
                if (more) sn = span(g0 + 64);
                uint32_t w[kChunkWords];
#ifdef FCS_SPAN_B32   // measurement-only: 25 dword reads at the window's 4-B address (bank conflicts)
                if (!cur.rare) {
                    const int x = cur.valid ? (int)(cur.cstart - (int64_t)sp.src) : 0;
                    const uint32_t r = (uint32_t)x & 3u;
                    const uint8_t *wp = slot + (x & ~3);
                    uint32_t d[kChunkWords + 1];
                    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
                    for (int q = 0; q < kChunkWords; q++) d[q] = *reinterpret_cast<const uint32_t *>(wp + 4 * q);
                    {
                        const uint8_t *a24 = wp + 4 * kChunkWords, *lim = slot + kDmaItemBytes - 4;
                        d[kChunkWords] = *reinterpret_cast<const uint32_t *>(a24 < lim ? a24 : lim);
                    }
                    __builtin_amdgcn_s_waitcnt(0xC07F);
#pragma unroll
                    for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], r);
                } else
#endif
                if (!cur.rare) {
                    // the window at its byte offset x in the slot (x >= -95: a front window reaching
                    // before the arena start reads LDS below the slot, bytes that get masked), read
                    // as seven 16-B pieces from x rounded down to 16 B: packed windows sit at 64..96-B
                    // strides, where ds_read_b32 would put 16-32 lanes on one bank (25 reads), and
                    // ds_read_b128 8-16 lanes on one 16-B group (7 reads; tools/microbench/lds_pat.hip)
                    const int x = cur.valid ? (int)(cur.cstart - (int64_t)sp.src) : 0;
                    const uint8_t *wp = slot + (x & ~15);
                    u32x4 q[7];
                    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the item's span has landed
#pragma unroll
                    for (int i = 0; i < 6; i++) q[i] = *reinterpret_cast<const u32x4 *>(wp + 16 * i);
                    {   // the 7th piece matters only when x is not 16-B aligned, and then lies in the slot
                        const uint8_t *a6 = wp + 96, *lim = slot + kDmaItemBytes - 16;
                        q[6] = *reinterpret_cast<const u32x4 *>(a6 < lim ? a6 : lim);
                    }
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next span
                    uint32_t d[28];
#pragma unroll
                    for (int i = 0; i < 7; i++) {
                        d[4 * i] = q[i].x;
                        d[4 * i + 1] = q[i].y;
                        d[4 * i + 2] = q[i].z;
                        d[4 * i + 3] = q[i].w;
                    }
                    // realign: dword shift s = (x >> 2) & 3 in two select stages, then the byte shift.
                    // The selects are v_perm (whole dword from either source): written as ?: the
                    // compiler turns the stages into an indexed array in scratch memory.
#ifdef FCS_SPAN_ABL_NOALIGN   // measurement-only: no realignment (wrong FCS unless x is 16-B aligned)
#pragma unroll
                    for (int i = 0; i < kChunkWords; i++) w[i] = d[i];
#else
                    const uint32_t p1 = (x & 4) ? 0x07060504u : 0x03020100u, p2 = (x & 8) ? 0x07060504u : 0x03020100u;
#pragma unroll
                    for (int i = 0; i < 26; i++) d[i] = __builtin_amdgcn_perm(d[i + 2], d[i], p2);
#pragma unroll
                    for (int i = 0; i < 25; i++) d[i] = __builtin_amdgcn_perm(d[i + 1], d[i], p1);
                    const uint32_t r = (uint32_t)x & 3u;
#pragma unroll
                    for (int i = 0; i < kChunkWords; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], r);
#endif
                } else {   // register loads (with the arena-edge shift)
                    Chunk ch;
                    issue_any<false>(p, cur.cstart, cur.valid && cur.zr < kChunkBytes, ch);
                    fd_chunk_words(ch, w);
                    __builtin_amdgcn_s_waitcnt(0x0F70);   // and a span DMA issued for this item, if any
                }
                if (more && !sn.rare) span_dma(slot, sn, lane);
                {
#ifdef FCS_SPAN_NOCRC   // measurement-only build: the span DMA, reads and dealing without the CRC work
                    uint32_t v = cur.c;
#pragma unroll
                    for (int i = 0; i < kChunkWords; i++) v ^= w[i];
#else
                    // lanes past the window's chunks and the dummy chunk of an empty frame (zr = 96) are discarded
                    const uint32_t own = fd_value(lds, w, cur.zr, cur.zr < kChunkBytes ? cur.zr : 0,
                                                  cur.valid ? fd_inv(lds, cur.zr) : 0u, B, SEL);
                    const uint32_t v = fd_chunk_shift(lds, own, cur.c & 15u);
#endif
                    if (cur.valid && v) atomicXor(reinterpret_cast<uint32_t *>(lds + fd_acc_addr(wave, (uint32_t)cur.src)), v);
                }
                if (more) prep(g0 + 64, sn, cur);
                sp = sn;
            }
        }

        // ---- frames over 1536 B: 16 lanes each, 4 per item, segment by segment (register loads) ----
        const uint64_t xmask = __ballot(multi);
        const uint32_t nx = (uint32_t)__popcll(xmask);
        if (nx) {
            const uint32_t rx = __builtin_amdgcn_mbcnt_hi((uint32_t)(xmask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)xmask, 0u));
            if (multi) mlist[rx] = (uint8_t)lane;
            wave_lds_sync();
            for (uint32_t t = 0; t < nx; t += 4) {
                const uint32_t rnk = t + (uint32_t)(lane >> 4);
                const bool valid = rnk < nx;
                const int src = valid ? (int)mlist[rnk] : 0;
                const uint64_t Eq = ((uint64_t)(uint32_t)__shfl((int)Ehi, src) << 32) | (uint32_t)__shfl((int)Elo, src);
                const uint32_t Lq = (uint32_t)__shfl((int)L, src);
                const uint32_t m = valid ? (Lq + (kSegBytes - 1)) / kSegBytes : 0u;
                uint32_t s = 0;
                for (uint32_t q = 0; __any(q < m); q++) {
                    const bool on = q < m;
                    const int64_t cstart = (int64_t)Eq - (int64_t)kSegBytes * (int64_t)(m - 1 - q) -
                                           (int64_t)kChunkBytes * (j + 1);
                    const int zr = (on && q == 0) ? clamp_zr((int64_t)(Eq - Lq) - cstart) : (on ? -1 : kChunkBytes);
                    Chunk cc;
                    issue_any<false>(p, cstart, on && zr < kChunkBytes, cc);
                    uint32_t w[kChunkWords];
                    fd_chunk_words(cc, w);
                    const uint32_t r = fd_value(lds, w, zr, on ? zr : 0, (on && q == 0) ? fd_inv(lds, zr) : 0u, B, SEL);
                    s = on ? (q == 0 ? r : fd_jump(lds, s, r)) : s;
                }
                const uint32_t v = row_xor(fd_chunk_shift(lds, s, (uint32_t)j));
                if (valid && j == 15) *reinterpret_cast<uint32_t *>(lds + fd_acc_addr(wave, (uint32_t)src)) = v;
            }
        }

        // ---- one coalesced store per window; clear the accumulators ----
        wave_lds_sync();
        uint32_t *accp = reinterpret_cast<uint32_t *>(lds + acc_lane);
        const uint32_t a = *accp;
        emit<kDmaBad>(p, lds, act, f, L ? ~a : 0u);
        *accp = 0u;
        win = nwin;
    }
    flush_bad<kDmaBad>(p, lds);
}
#endif  // FCS_SPAN

// Counter-based byte generator: 8-byte word q of the stream = splitmix64(seed + q).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t *p, uint64_t bytes,
                                                            uint64_t seed, uint64_t off) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nth = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t head = (8 - (off & 7)) & 7;   // bytes before the first aligned stream word
    for (uint64_t i = tid; i < head && i < bytes; i += nth) {
        const uint64_t q = off + i;
        p[i] = (uint8_t)(splitmix64(seed + (q >> 3)) >> (8 * (q & 7)));
    }
    if (bytes <= head) return;
    const uint64_t body_words = (bytes - head) / 8;
    const uint64_t w0 = (off + head) >> 3;
    uint8_t *pb = p + head;
    const bool al8 = (((uintptr_t)pb) & 7) == 0;
    for (uint64_t i = tid; i < body_words; i += nth) {
        const uint64_t v = splitmix64(seed + w0 + i);
        if (al8) {
            reinterpret_cast<uint64_t *>(pb)[i] = v;
        } else {
#pragma unroll
            for (int b = 0; b < 8; b++) pb[8 * i + b] = (uint8_t)(v >> (8 * b));
        }
    }
    for (uint64_t i = head + body_words * 8 + tid; i < bytes; i += nth) {
        const uint64_t q = off + i;
        p[i] = (uint8_t)(splitmix64(seed + (q >> 3)) >> (8 * (q & 7)));
    }
}

// Pure read stream: 16 B per lane per load, 4 loads in flight, XOR folded to one word per thread.
__global__ __launch_bounds__(256) void read_stream_kernel(const u32x4 *__restrict__ p, uint64_t n16,
                                                          uint32_t *sink) {
    uint32_t acc = 0;
    const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t pb = (uint64_t)p;
    for (; i + 3 * st < n16; i += 4 * st) {
        const u32x4 a = gload<u32x4>(pb + 16 * i), b = gload<u32x4>(pb + 16 * (i + st)),
                    c = gload<u32x4>(pb + 16 * (i + 2 * st)), e = gload<u32x4>(pb + 16 * (i + 3 * st));
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ e.x ^ e.y ^
               e.z ^ e.w;
    }
    for (; i < n16; i += st) {
        const u32x4 a = p[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;   // keep the loads live; practically never stores
}

// Completion signal for small host batches: launched behind the FCS kernel on the same stream,
// it stores `v` into a device-mapped host word, on which the host spins instead of synchronising
// the stream (cuts the hipStreamSynchronize wake-up from the round trip).
__global__ void signal_kernel(uint64_t *flag, uint64_t v) {
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The single-frame tables (7 KiB) into LDS: every load issued before the first store, so the
// wave waits for one memory latency instead of seven in a row.
__device__ __forceinline__ void stage_one_blob(uint32_t *t, const uint32_t *blob, int lane) {
    constexpr int kIters = kOneBlobWords / 4 / 64;
    static_assert(kOneBlobWords % 256 == 0, "one 16-byte piece per lane per step");
    u32x4a4 v[kIters];
#pragma unroll
    for (int k = 0; k < kIters; k++) v[k] = reinterpret_cast<const u32x4a4 *>(blob)[lane + 64 * k];
#pragma unroll
    for (int k = 0; k < kIters; k++) reinterpret_cast<u32x4a4 *>(t)[lane + 64 * k] = v[k];
}

// Drop-in ether_fcs for one frame (fcs_launch.hpp OneArgs). The frame arrives in the kernel
// arguments, right-aligned in a 1536-byte window with zeros in front: from a zero register,
// leading zeros change nothing, and the all-ones start of the real CRC is added back as
// kinit = A_len(0xFFFFFFFF) (the register update is affine: R(s, M) = A_len(s) ^ R(0, M)).
// Lane j runs six slice-by-4 steps over window bytes [24j, 24j + 24) from a zero register; a
// six-level tree then joins neighbouring lane groups, the earlier one advanced by A_{24 * 2^k}.
// Lane 0 stores (seq << 32) | FCS into a mapped host word with one system-scope store, which
// is also the completion signal the host spins on: no staging copy, no second launch.
__device__ __forceinline__ uint32_t one_step(const uint32_t *t, uint32_t x, uint32_t wn) {
    return xor3(xor3(t[768 + (x & 0xFFu)], t[512 + ((x >> 8) & 0xFFu)], t[256 + ((x >> 16) & 0xFFu)]),
                t[x >> 24], wn);
}

__global__ __launch_bounds__(64) void fcs_one_kernel(OneArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t t[kOneBlobWords];
    const int lane = threadIdx.x;
#ifndef FCS_ONE_NOBLOB   // measurement-only build: tables not staged (wrong FCS; timing only)
    stage_one_blob(t, a.blob, lane);
#endif
    // the window words straight from the kernel-argument segment (no private copy of `a`)
    typedef const __attribute__((address_space(4))) uint32_t karg_u32;
    karg_u32 *dw = reinterpret_cast<karg_u32 *>(
        (const __attribute__((address_space(4))) uint8_t *)__builtin_amdgcn_kernarg_segment_ptr() +
        offsetof(OneArgs, data));
    uint32_t w[6];
#ifdef FCS_ONE_NOARG   // measurement-only build: the frame words not read (wrong FCS; timing only)
#pragma unroll
    for (int q = 0; q < 6; q++) w[q] = lane * 6 + q;
    (void)dw;
#else
#pragma unroll
    for (int q = 0; q < 6; q++) w[q] = dw[lane * 6 + q];
#endif
    __syncthreads();
    uint32_t x = w[0];
#pragma unroll
    for (int i = 0; i < 6; i++) x = one_step(t, x, i < 5 ? w[i + 1] : 0u);
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const uint32_t *nt = t + 1024 + k * 128;
        uint32_t y = x;
        if (!(lane & (1 << k))) {   // the earlier group: advance it past the later one's bytes
            uint32_t r[8];
#pragma unroll
            for (int q = 0; q < 8; q++) r[q] = nt[q * 16 + ((x >> (4 * q)) & 15u)];
            y = xor9(r, 0u);
        }
        x = y ^ (uint32_t)__shfl_xor((int)y, 1 << k);
    }
    if (lane == 0)
        __hip_atomic_store(a.flag, ((uint64_t)a.seq << 32) | (uint64_t)(uint32_t)~(x ^ a.kinit), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// One wave's frame of at most kOneBytes bytes ending at `end` and starting at `start`, read from
// (mapped) memory: the same window, lane chain and tree as fcs_one_kernel. The wave first copies
// the 16-byte blocks that hold the frame into its LDS window with coalesced 16-byte loads (host
// memory over PCIe wants few, wide requests), then every lane takes its 24 bytes from there.
// Blocks start with the one holding `start` and end with the one holding end - 1: no byte of
// another page is touched (the frame may open or close its allocation). The realignment's last
// LDS dword may reach past the copied bytes; those bytes lie beyond the lane's 24 and are unused.
constexpr uint32_t kOneWinBytes = kOneBytes + 32;   // per-wave LDS window (16-B aligned base)

// The tables (blob, staged into t) and the frame are fetched together: every load of both is
// issued before the first LDS store, so the table latency hides under the frame's PCIe reads.
__device__ __forceinline__ uint32_t one_frame_reg(uint32_t *t, const uint32_t *blob, uint8_t *win, uint64_t start,
                                                  uint64_t end, int lane) {
    const uint64_t wbase = end - kOneBytes;            // window byte 0 (may precede the frame)
    const uint64_t g0 = wbase & ~15ull;                // LDS byte 0 <-> this address
    const uint64_t b0 = (start > wbase ? start : wbase) & ~15ull;
    const uint64_t b1 = (end + 15) & ~15ull;           // one past the last block to load
    constexpr int kTab = kOneBlobWords / 4 / 64;
    constexpr int kBlk = (kOneWinBytes / 16 + 63) / 64;
    u32x4a4 tv[kTab], fv[kBlk];
#pragma unroll
    for (int k = 0; k < kTab; k++) tv[k] = reinterpret_cast<const u32x4a4 *>(blob)[lane + 64 * k];
#pragma unroll
    for (int k = 0; k < kBlk; k++) {
        const uint64_t a = b0 + 16 * (uint64_t)(lane + 64 * k);
        if (a < b1) fv[k] = gload<u32x4a4>(a);
    }
#pragma unroll
    for (int k = 0; k < kTab; k++) reinterpret_cast<u32x4a4 *>(t)[lane + 64 * k] = tv[k];
#pragma unroll
    for (int k = 0; k < kBlk; k++) {
        const uint64_t a = b0 + 16 * (uint64_t)(lane + 64 * k);
        if (a < b1) *reinterpret_cast<u32x4a4 *>(win + (a - g0)) = fv[k];
    }
    __syncthreads();
    const int64_t c = (int64_t)wbase + 24 * lane;      // this lane's window bytes [c, c + 24)
    uint32_t w[6] = {0, 0, 0, 0, 0, 0};
    if (c + 24 > (int64_t)start) {
        const uint32_t p = (uint32_t)((uint64_t)c - g0);
        const uint32_t r = p & 3u;
        uint32_t d[7];
#pragma unroll
        for (int q = 0; q < 7; q++) d[q] = *reinterpret_cast<const uint32_t *>(win + (p & ~3u) + 4 * q);
        const int zr = (int)((int64_t)start - c);      // window bytes before the frame: masked
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const uint32_t v = __builtin_amdgcn_alignbyte(d[i + 1], d[i], r);
            int z = zr - 4 * i;
            z = z < 0 ? 0 : (z > 4 ? 4 : z);
            w[i] = v & (uint32_t)(0xFFFFFFFFull << (8 * z));
        }
    }
    wave_lds_sync();                                   // window reads done before the next frame's copy
    uint32_t x = w[0];
#pragma unroll
    for (int i = 0; i < 6; i++) x = one_step(t, x, i < 5 ? w[i + 1] : 0u);
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const uint32_t *nt = t + 1024 + k * 128;
        uint32_t y = x;
        if (!(lane & (1 << k))) {
            uint32_t r8[8];
#pragma unroll
            for (int q = 0; q < 8; q++) r8[q] = nt[q * 16 + ((x >> (4 * q)) & 15u)];
            y = xor9(r8, 0u);
        }
        x = y ^ (uint32_t)__shfl_xor((int)y, 1 << k);
    }
    return x;
}

// A small-batch frame's result: RX verify writes ok[f] (the frame carries its trailer; it checks
// iff the residue shows), TX writes the FCS little-endian right after the frame
// (src/linux/ether.c:263). Then the frame counts itself done; the batch's last frame stores seq.
__device__ __forceinline__ void small_finish(uint32_t fcs, uint8_t *ok, uint32_t f, uint64_t start, uint32_t L,
                                             int lane, unsigned long long *count, uint64_t count_base, uint32_t n,
                                             uint64_t *flag, uint64_t seq) {
    if (ok) {
        if (lane == 0) ok[f] = (L >= 4 && fcs == 0x2144DF1Cu) ? 1 : 0;
    } else if (lane < 4) {
        *reinterpret_cast<__attribute__((address_space(1))) uint8_t *>(start + L + lane) = (uint8_t)(fcs >> (8 * lane));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // this frame's result has reached host memory
    if (lane == 0) {
        const uint64_t done = __hip_atomic_fetch_add(count, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (done == count_base + n - 1)   // the batch's last frame
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// One workgroup (one wave) per frame, so the frames' PCIe reads come from as many CUs: one CU
// reading 16 frames of host memory took 17.7 us, against 10.6 us for one. Each wave writes its
// FCS into the frame, makes it visible system-wide and counts itself done on a device counter;
// the last one to finish stores `seq` into the mapped completion word.
__global__ __launch_bounds__(64) void fcs_tx_small_kernel(TxSmallArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t t[kOneBlobWords];
    __shared__ __attribute__((aligned(16))) uint8_t win[kOneWinBytes];
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    typedef const __attribute__((address_space(4))) uint8_t karg_u8;
    karg_u8 *ka = (karg_u8 *)__builtin_amdgcn_kernarg_segment_ptr();
    const uint64_t o = *(const __attribute__((address_space(4))) uint64_t *)(ka + offsetof(TxSmallArgs, off) + 8 * f);
    const uint32_t L = *(const __attribute__((address_space(4))) uint32_t *)(ka + offsetof(TxSmallArgs, len) + 4 * f);
    const uint32_t ki = *(const __attribute__((address_space(4))) uint32_t *)(ka + offsetof(TxSmallArgs, kinit) + 4 * f);
    const uint64_t start = (uint64_t)a.base + o;
    const uint32_t x = one_frame_reg(t, a.blob, win, start, start + L, lane);
    small_finish(~(x ^ ki), a.ok, f, start, L, lane, a.count, a.count_base, a.n, a.flag, a.seq);
}

__global__ __launch_bounds__(64) void fcs_small_list_kernel(ListArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t t[kOneBlobWords];
    __shared__ __attribute__((aligned(16))) uint8_t win[kOneWinBytes];
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    const uint64_t o = a.off[f];      // one mapped read each (uniform address)
    const uint32_t L = a.len[f];
    const uint32_t ki = a.kinit[L < kOneBytes ? L : kOneBytes];
    const uint64_t start = (uint64_t)a.base + o;
    const uint32_t x = one_frame_reg(t, a.blob, win, start, start + L, lane);
    small_finish(~(x ^ ki), a.ok, f, start, L, lane, a.count, a.count_base, a.n, a.flag, a.seq);
}

// TX mode helper: after the FCS kernel wrote crc[i], store it little-endian after each frame.
__global__ __launch_bounds__(256) void tx_store_kernel(uint8_t *base, uint64_t stride,
                                                       const uint32_t *len, const uint32_t *crc,
                                                       uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t *q = base + i * stride + len[i];
    const uint32_t c = crc[i];
    q[0] = (uint8_t)c;
    q[1] = (uint8_t)(c >> 8);
    q[2] = (uint8_t)(c >> 16);
    q[3] = (uint8_t)(c >> 24);
}

// ---- host-side launchers (the engine TU never names the kernels) ----
hipError_t launch_fcs(bool var, bool windowed, const KParams &p, int grid, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    const bool tiny = fixed_tiny(p);
    const bool single = !var && fixed_single(p);
    // fixed_threads(p) (fcs_launch.hpp) picks the workgroup size; the host sized the grid with it
#define FCS_LAUNCH(V, T, S) \
    hipLaunchKernelGGL((fcs_kernel<V, T, S, kWgThreads>), dim3(grid), dim3(kWgThreads), 0, st, p)
    if (var) {
        // windowed: throughput form (64-frame windows per wave, chunks dealt flat to the lanes);
        // otherwise one quarter-wave per frame, every frame in flight at once (small batches)
        if (!windowed) {
            if (tiny) FCS_LAUNCH(true, true, false);
            else FCS_LAUNCH(true, false, false);
        } else if (tiny) {
#ifdef FCS_VAR_HALFUNIT   // measurement-only build: the half-unit windowed kernel it replaced
            hipLaunchKernelGGL((fcs_var_kernel<true>), dim3(grid), dim3(kWgThreads), 0, st, p);
#else
            hipLaunchKernelGGL((fcs_flat_kernel<true>), dim3(grid), dim3(kWgThreads), 0, st, p);
#endif
        } else {
#if defined(FCS_VAR_HALFUNIT)
            hipLaunchKernelGGL((fcs_var_kernel<false>), dim3(grid), dim3(kWgThreads), 0, st, p);
#elif defined(FCS_FLATDMA)   // measurement-only build: per-lane window DMA (rejected)
            hipLaunchKernelGGL(fcs_flatdma_kernel, dim3(grid), dim3(kWgThreads), 0, st, p);
#else
#ifdef FCS_FLAT2
            if (var_flat2(p)) hipLaunchKernelGGL(fcs_flat2_kernel<kFlat2Threads>, dim3(2 * grid), dim3(kFlat2Threads), 0, st, p);
            else
#endif
#ifdef FCS_SPAN   // measurement-only build: span DMA (rejected)
            if (var_span(p)) hipLaunchKernelGGL(fcs_span_kernel, dim3(grid), dim3(kWgThreads), 0, st, p);
            else
#endif
            hipLaunchKernelGGL((fcs_flat_kernel<false>), dim3(grid), dim3(kWgThreads), 0, st, p);
#endif
        }
    } else if (fixed_segil(p)) {
        hipLaunchKernelGGL(fcs_segil_kernel, dim3(grid), dim3(kSegilThreads), 0, st, p);
#ifdef FCS_DMASEG
    } else if (!tiny && fixed_dmaseg(p)) {
        if (p.zmax <= 8) hipLaunchKernelGGL((fcs_dmaseg_kernel<2>), dim3(grid), dim3(kDmaWgThreads), 0, st, p);
        else hipLaunchKernelGGL((fcs_dmaseg_kernel<kSingleMaskWords>), dim3(grid), dim3(kDmaWgThreads), 0, st, p);
#endif
    } else if (!tiny && fixed_dma(p)) {
        if (p.zmax <= 8) hipLaunchKernelGGL((fcs_dma_kernel<2, false>), dim3(grid), dim3(kDmaWgThreads), 0, st, p);
        else hipLaunchKernelGGL((fcs_dma_kernel<kSingleMaskWords, false>), dim3(grid), dim3(kDmaWgThreads), 0, st, p);
    } else if (tiny) {
        if (single) FCS_LAUNCH(false, true, true);
        else FCS_LAUNCH(false, true, false);
    } else if (single) {
#ifdef FCS_OLD_SINGLE   // measurement-only build: generic kernel's SINGLE instantiation
        FCS_LAUNCH(false, false, true);
#else
        hipLaunchKernelGGL(fcs_single_kernel, dim3(grid), dim3(kFixedWgThreads), 0, st, p);
#endif
    } else if (fixed_threads(p) == kFixedWgThreads) {
        hipLaunchKernelGGL((fcs_kernel<false, false, false, kFixedWgThreads>), dim3(grid), dim3(kFixedWgThreads), 0, st, p);
    } else {
        FCS_LAUNCH(false, false, false);
    }
#undef FCS_LAUNCH
    return hipGetLastError();
}

hipError_t launch_signal(uint64_t *flag, uint64_t v, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, st, flag, v);
    return hipGetLastError();
}

hipError_t launch_fill(void *p, uint64_t bytes, uint64_t seed, uint64_t off, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    uint64_t words = bytes / 8 + 1;
    int grid = (int)((words + 255) / 256);
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, seed, off);
    return hipGetLastError();
}

hipError_t launch_read_stream(const void *p, uint64_t bytes, uint32_t *sink, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    hipLaunchKernelGGL(read_stream_kernel, dim3(8192), dim3(256), 0, st, (const u32x4 *)p, bytes / 16, sink);
    return hipGetLastError();
}

hipError_t launch_dma_stream(const KParams &p, int grid, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    hipLaunchKernelGGL((fcs_dma_kernel<2, true>), dim3(grid), dim3(kDmaWgThreads), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_one(const OneArgs &a, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    hipLaunchKernelGGL(fcs_one_kernel, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_tx_small(const TxSmallArgs &a, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    hipLaunchKernelGGL(fcs_tx_small_kernel, dim3(a.n), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_small_list(const ListArgs &a, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    hipLaunchKernelGGL(fcs_small_list_kernel, dim3(a.n), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_tx_store(uint8_t *base, uint64_t stride, const uint32_t *len, const uint32_t *crc,
                           uint64_t n, hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(tx_store_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, base, stride, len, crc, n);
    return hipGetLastError();
}

}  // namespace fcs
