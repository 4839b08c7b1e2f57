// inet_kernel.hip — batched Internet checksums (RFC 1071 one's-complement sums) for gfx950.
//
// Serves SURVEY.md §8f row 3: the per-packet byte loops of nstack's
//   ip_checksum   /root/reference/src/ip.c:39-62     (IP headers; ICMP via src/icmp.c:42,74)
//   tcp_checksum  /root/reference/src/tcp.c:167-213  (12-byte pseudo header, then the segment)
//   udp_checksum  /root/reference/src/udp.c:136-174  (the segment, then the pseudo header)
// as one launch over many packets; out[i] is bit-identical to the reference function's return
// value (a host-order u16 whose memory bytes are the on-wire checksum).
//
// Arithmetic. All three are one's-complement sums of little-endian 16-bit words (the reference
// memcpy's host-order words; RFC 1071's byte-order independence makes that the byte-swapped
// checksum, which is exactly what it stores). Because 2^16 == 1 (mod 0xffff), a sum of 32-bit
// words folded to 16 bits has the same residue, so each lane adds whole dwords of its 16-byte
// chunks into a 64-bit register (v_add_co / v_addc per dword) and only the 16-lane total is
// folded. A packet starting at an odd address pairs its bytes the other way round against the
// aligned memory words: the memory-aligned sum M then satisfies P == 256*M (mod 0xffff), i.e.
// P = swap16(fold(M)). The exact-zero case is kept apart from 0xffff (fold never maps a
// nonzero sum to 0), because ip/tcp start their accumulator at 0xffff (ip.c:42, tcp.c:172):
// the only input where that differs from a zero start is all-zero data (return 0x0000).
//
// Kernels (launch_inet picks one; results are identical): small batches a QUARTER-WAVE (16 lanes)
// per packet (inet_kernel: lane j loads the packet's aligned 16-byte chunks j, j+16, ..., six in
// flight per round; the 16 lane sums added with 4 DPP steps; lane 0 adds the pseudo header and
// init, folds, complements and stores); large batches the flat chunk stream (inet_flat_kernel),
// short fixed packets one lane per packet (inet_short_kernel), fixed strides four packets per LDS-DMA
// slot (inet_dma_kernel) and packed variable windows through LDS (inet_stream_kernel). No tables:
// HBM read bandwidth is the roofline.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dispenser.hpp"
#include "inet_launch.hpp"
#include "wave_sync.hpp"

namespace inet {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kGroup = 16;       // lanes per packet
constexpr int kRound = 6;        // chunks per lane per round
constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ T gload(uint64_t addr) {
#ifdef FCS_NT   // measurement-only build: non-temporal (nt) packet loads
    return __builtin_nontemporal_load(reinterpret_cast<const __attribute__((address_space(1))) T *>(addr));
#else
    return *reinterpret_cast<const __attribute__((address_space(1))) T *>(addr);
#endif
}

__device__ __forceinline__ uint32_t swap16(uint32_t x) { return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu); }

// End-around-carry fold to [0, 0xffff]; 0 only for x == 0.
__device__ __forceinline__ uint32_t fold64(uint64_t x) {
    uint64_t y = (x & 0xffffffffull) + (x >> 32);
    y = (y & 0xffffu) + (y >> 16);
    y = (y & 0xffffu) + (y >> 16);
    return (uint32_t)((y & 0xffffu) + (y >> 16));
}

// Sum over a 16-lane row; every lane ends with the row's sum.
__device__ __forceinline__ uint32_t row_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    return v;
}

// Byte mask of dword d of a chunk from a 16-bit keep mask (bit b = keep byte b of the chunk).
__device__ __forceinline__ uint32_t byte_mask(uint32_t keep16, int d) {
    const uint32_t b4 = (keep16 >> (4 * d)) & 0xfu;
    return ((b4 * 0x00204081u) & 0x01010101u) * 0xffu;
}

// Pseudo-header contribution and accumulator start of each mode (exact integers, summed in the
// little-endian word domain the reference uses).
template <int MODE>
__device__ __forceinline__ uint32_t pseudo_sd(uint32_t s, uint32_t d, uint32_t len) {
    const uint32_t l16 = swap16(len & 0xffffu);   // htons(len): size_t truncated to 16 bits
    if (MODE == kIp) return 0xffffu;              // acc = 0xffff (src/ip.c:42)
    if (MODE == kTcp)                             // acc = 0xffff; {htonl(src), htonl(dst), 0, 6, htons(len)}
        return 0xffffu + swap16(s >> 16) + swap16(s & 0xffffu) + swap16(d >> 16) + swap16(d & 0xffffu) +
               0x0600u + l16;                     // (src/tcp.c:172-195)
    // udp: sum = 0; raw in_addr_t halves, htons(IPPROTO_UDP), htons(length) (src/udp.c:146,160-167)
    return (s & 0xffffu) + (s >> 16) + (d & 0xffffu) + (d >> 16) + 0x1100u + l16;
}

template <int MODE>
__device__ __forceinline__ uint32_t pseudo(const IParams &p, uint64_t i, uint32_t len) {
    if (MODE == kIp) return pseudo_sd<MODE>(0u, 0u, len);
    return pseudo_sd<MODE>(p.addr[2 * i], p.addr[2 * i + 1], len);
}

// One packet's geometry.
struct Pkt {
    uint64_t start, c0;   // first byte; its 16-byte aligned chunk
    uint32_t len, nch;    // bytes; 16-byte chunks touched (0 for an empty packet)
};

template <bool VAR>
__device__ __forceinline__ Pkt packet(const IParams &p, uint64_t i, uint64_t off, uint32_t len) {
    Pkt k;
    k.start = VAR ? p.base + off : p.base + i * p.stride;
    k.len = VAR ? len : p.flen;
    k.c0 = k.start & ~15ull;
    const uint64_t end = k.start + k.len;
    k.nch = k.len ? (uint32_t)((((end + 15) & ~15ull) - k.c0) >> 4) : 0u;
    return k;
}

// Issue the loads of round k0 of packet k. Lanes past the packet's last chunk re-read that chunk
// (an L1/L2 hit; zeroed in accumulate): unconditional loads from one base keep the round's
// six loads back to back. An empty packet loads nothing.
__device__ __forceinline__ void issue(const Pkt &k, uint32_t k0, uint32_t lane, u32x4 (&v)[kRound]) {
    if (k.nch == 0) return;
#pragma unroll
    for (int j = 0; j < kRound; j++) {
        const uint32_t c = k0 + lane + kGroup * j;
        v[j] = gload<u32x4>(k.c0 + 16ull * (c < k.nch ? c : k.nch - 1));
    }
}

// Add round k0 of packet k into acc (only the packet's first and last chunk are masked).
__device__ __forceinline__ void accumulate(const Pkt &k, uint32_t k0, uint32_t lane, const u32x4 (&v)[kRound],
                                           uint64_t &acc) {
#pragma unroll
    for (int j = 0; j < kRound; j++) {
        const uint32_t c = k0 + lane + kGroup * j;
        if (c >= k.nch) continue;
        u32x4 w = v[j];
        if (c == 0 || c + 1 == k.nch) {   // edge chunks: keep bytes in [start, end)
            const uint64_t ca = k.c0 + 16ull * c, end = k.start + k.len;
            const uint32_t lo = k.start > ca ? (uint32_t)(k.start - ca) : 0u;
            const uint32_t hi = end - ca < 16 ? (uint32_t)(end - ca) : 16u;
            const uint32_t keep = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
            w.x &= byte_mask(keep, 0);
            w.y &= byte_mask(keep, 1);
            w.z &= byte_mask(keep, 2);
            w.w &= byte_mask(keep, 3);
        }
        acc += (uint64_t)w.x + w.y;
        acc += (uint64_t)w.z + w.w;
    }
}

// Software-pipelined per group of 16 lanes: while packet i is reduced, the loads of the group's
// next packet are in flight and (variable batches) the offset/length of the one after that.
template <bool VAR, int MODE>
__global__ __launch_bounds__(kThreads) void inet_kernel(IParams p) {
    const uint32_t lane = threadIdx.x & (kGroup - 1);
    const uint64_t ngrp = ((uint64_t)gridDim.x * kThreads) / kGroup;
    uint64_t i = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) / kGroup;
    if (i >= p.n) return;   // whole groups leave together
    auto meta_off = [&](uint64_t q) -> uint64_t { return VAR && q < p.n ? p.off[q] : 0ull; };
    auto meta_len = [&](uint64_t q) -> uint32_t { return VAR && q < p.n ? p.len[q] : 0u; };
    Pkt cur = packet<VAR>(p, i, meta_off(i), meta_len(i));
    uint64_t noff = meta_off(i + ngrp);
    uint32_t nlen = meta_len(i + ngrp);
    u32x4 va[kRound], vb[kRound];
    issue(cur, 0, lane, va);
    // one packet: its round-0 chunks are in `v`; the next packet's go into `w`. Returns false
    // after the group's last packet. (Two copies with the buffers swapped: no register moves.)
    auto step = [&](u32x4 (&v)[kRound], u32x4 (&w)[kRound]) -> bool {
        const uint64_t inext = i + ngrp;
        const bool more = inext < p.n;
        Pkt nxt = packet<VAR>(p, inext, noff, nlen);
        if (!more) nxt.nch = 0;
        noff = meta_off(inext + ngrp);   // two packets ahead
        nlen = meta_len(inext + ngrp);
        issue(nxt, 0, lane, w);          // one packet ahead
        uint64_t acc = 0;
        accumulate(cur, 0, lane, v, acc);
        for (uint32_t k0 = kGroup * kRound; k0 < cur.nch; k0 += kGroup * kRound) {   // > 1536 B
            issue(cur, k0, lane, v);
            accumulate(cur, k0, lane, v, acc);
        }
        const uint32_t s = fold64(row_sum(fold64(acc)));   // <= 16 * 0xffff before the outer fold
        if (lane == 0) {
            const uint32_t m = (cur.start & 1) ? swap16(s) : s;   // odd start: P = swap16(fold(M))
            const uint32_t t = fold64((uint64_t)pseudo<MODE>(p, i, cur.len) + m);
            p.out[i] = (uint16_t)~t;
        }
        i = inext;
        cur = nxt;
        return more;
    };
    while (step(va, vb) && step(vb, va)) {
    }
}

// ---------------------------------------------------------------------------------------------
// Variable-length batches, flat chunk stream (inet_flat_kernel): a wave owns windows of 64
// consecutive packets. Packet i needs k = ceil(nch / 6) lane units of six 16-byte chunks (96 B,
// interleaved: unit u holds chunks u, u + k, ..., so the packet's lanes load coalesced rows);
// the window's units are numbered packet by packet and dealt to the lanes 64 at a time, so a
// 64-byte packet takes one lane instead of a 16-lane round. A lane finds its packet from
// frame-start marks (as fcs_flat_kernel), loads its six chunks, masks the packet's edge chunks,
// and adds its folded sum into the packet's LDS accumulator (ds_add_u64). The sum needs no
// position shift, so a packet of any length stays in the stream. Lane i finishes packet i at the
// end of the window (coalesced u16 stores).
// ---------------------------------------------------------------------------------------------
constexpr int kUnit = 6;   // 16-byte chunks per lane unit

// One window of 64 packets from w0 by the flat chunk stream (acc, mark: this wave's zeroed LDS
// arrays, left zeroed; list: its scratch).
template <bool VAR, int MODE>
__device__ __forceinline__ void flat_window(const IParams &p, uint64_t w0, int lane, unsigned long long *acc,
                                            uint8_t *mark, uint8_t *list) {
    const uint64_t i = w0 + lane;
    const bool act = i < p.n;
    const uint32_t len = act ? (VAR ? p.len[i] : p.flen) : 0u;
    const uint64_t start = act ? p.base + (VAR ? p.off[i] : i * p.stride) : 0ull;
    const uint64_t c0 = start & ~15ull;
    const uint32_t nch = len ? (uint32_t)((((start + len + 15) & ~15ull) - c0) >> 4) : 0u;
    const uint32_t k = (nch + kUnit - 1) / kUnit;
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
    if (k) list[rank] = (uint8_t)lane;
    wave_lds_sync();
    const uint32_t c0lo = (uint32_t)c0, c0hi = (uint32_t)(c0 >> 32);
    const uint32_t edges = (uint32_t)(start & 15) | ((uint32_t)((start + len) & 15) << 8);

    for (uint32_t g0 = 0; g0 < K; g0 += 64) {
        // a long packet spans any number of items, so marks are cleared after use (not tagged)
        const bool starts = k && P >= g0 && P < g0 + 64;
        if (starts) mark[P - g0] = 1;
        wave_lds_sync();
        const uint32_t before = (uint32_t)__popcll(__ballot(k && P < g0));
        const uint64_t M = __ballot(mark[lane] != 0);
        wave_lds_sync();
        if (starts) mark[P - g0] = 0;
        const uint32_t g = g0 + (uint32_t)lane;
        const bool valid = g < K;
        const uint32_t rk = before + (uint32_t)__popcll(M & ((2ull << lane) - 1ull)) - 1u;
        const int src = valid ? (int)list[rk & 63u] : 0;
        const uint64_t cb = ((uint64_t)(uint32_t)__shfl((int)c0hi, src) << 32) | (uint32_t)__shfl((int)c0lo, src);
        const uint32_t nc = (uint32_t)__shfl((int)nch, src);
        const uint32_t Pg = (uint32_t)__shfl((int)P, src);
        const uint32_t eg = (uint32_t)__shfl((int)edges, src);
        // unit u of a k-unit packet holds chunks u, u + k, ..., u + 5k: load q of the packet's k
        // lanes reads k consecutive chunks (coalesced), the sum does not care about the order
        const uint32_t u = g - Pg, kg = (nc + kUnit - 1) / kUnit;
        if (valid) {
            u32x4 v[kUnit];
#pragma unroll
            for (int q = 0; q < kUnit; q++) {
                const uint32_t c = u + q * kg;
                v[q] = gload<u32x4>(cb + 16ull * (c < nc ? c : nc - 1));   // past the end: a cache hit, zeroed below
            }
            uint64_t s = 0;
#pragma unroll
            for (int q = 0; q < kUnit; q++) {
                const uint32_t c = u + q * kg;
                if (c >= nc) continue;
                u32x4 w = v[q];
                if (c == 0 || c + 1 == nc) {   // the packet's edge chunks: keep bytes in [start, end)
                    const uint32_t lo = c == 0 ? (eg & 0xffu) : 0u;
                    const uint32_t e15 = (eg >> 8) & 0xffu;
                    const uint32_t hi = (c + 1 == nc && e15) ? e15 : 16u;
                    const uint32_t keep = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
                    w.x &= byte_mask(keep, 0);
                    w.y &= byte_mask(keep, 1);
                    w.z &= byte_mask(keep, 2);
                    w.w &= byte_mask(keep, 3);
                }
                s += (uint64_t)w.x + w.y;
                s += (uint64_t)w.z + w.w;
            }
            const uint32_t f = fold64(s);   // 0 only for an all-zero unit
            if (f) atomicAdd(&acc[src], (unsigned long long)f);
        }
    }

    // ---- packet i: fold, odd-start swap, pseudo header and init, complement; clear state ----
    wave_lds_sync();
    const uint32_t m0 = fold64(acc[lane]);
    const uint32_t m = (start & 1) ? swap16(m0) : m0;   // odd start: P = swap16(fold(M))
    if (act) p.out[i] = (uint16_t)~fold64((uint64_t)pseudo<MODE>(p, i, len) + m);
    acc[lane] = 0ull;
    mark[lane] = 0;
}

template <bool VAR, int MODE>
__global__ __launch_bounds__(kThreads) void inet_flat_kernel(IParams p) {
    __shared__ unsigned long long acc_s[kThreads / 64][64];
    __shared__ uint8_t mark_s[kThreads / 64][64];
    __shared__ uint8_t list_s[kThreads / 64][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    acc_s[wave][lane] = 0ull;
    mark_s[wave][lane] = 0;
    const uint64_t GW = (uint64_t)gridDim.x * (kThreads / 64);
    for (uint64_t w0 = ((uint64_t)blockIdx.x * (kThreads / 64) + wave) * 64; w0 < p.n; w0 += GW * 64)
        flat_window<VAR, MODE>(p, w0, lane, acc_s[wave], mark_s[wave], list_s[wave]);
}

// Short packets (at most kShortMax bytes): the 16-B pieces a packet touches, and their sum.
constexpr uint32_t kShortMax = 64;
constexpr int kShortPieces = (int)(kShortMax + 15 + 15) / 16;   // 5

// Loads the pieces of the packet [start, start + L) (L >= 1): piece q of the packet's first 16-B
// boundary, or its last piece again past the end (a cache hit).
__device__ __forceinline__ void short_issue(uint64_t start, uint32_t L, u32x4 (&v)[kShortPieces]) {
    const uint64_t c0 = start & ~15ull;
    const uint32_t nch = (uint32_t)((((start + L + 15) & ~15ull) - c0) >> 4);
#pragma unroll
    for (int q = 0; q < kShortPieces; q++)
        v[q] = gload<u32x4>(c0 + 16ull * ((uint32_t)q < nch ? (uint32_t)q : nch - 1));
}

// The folded sum of the packet's bytes from its loaded pieces: edge pieces masked to
// [start, start + L), even- and odd-addressed bytes summed by v_dot4_u32_u8 (0 for L == 0).
__device__ __forceinline__ uint32_t short_sum(const u32x4 (&v)[kShortPieces], uint64_t start, uint32_t L) {
    const uint64_t c0 = start & ~15ull, end = start + L;
    const uint32_t nch = L ? (uint32_t)((((end + 15) & ~15ull) - c0) >> 4) : 0u;
    uint32_t E = 0, O = 0;
#pragma unroll
    for (int q = 0; q < kShortPieces; q++) {
        if ((uint32_t)q >= nch) break;
        u32x4 x = v[q];
        if (q == 0 || (uint32_t)q + 1 == nch) {   // edge pieces: keep bytes in [start, end)
            const uint64_t ca = c0 + 16ull * (uint32_t)q;
            const uint32_t lo = start > ca ? (uint32_t)(start - ca) : 0u;
            const uint32_t hi = end - ca < 16 ? (uint32_t)(end - ca) : 16u;
            const uint32_t keep = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
            x.x &= byte_mask(keep, 0);
            x.y &= byte_mask(keep, 1);
            x.z &= byte_mask(keep, 2);
            x.w &= byte_mask(keep, 3);
        }
        E = __builtin_amdgcn_udot4(x.x, 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(x.x, 0x01000100u, O, false);
        E = __builtin_amdgcn_udot4(x.y, 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(x.y, 0x01000100u, O, false);
        E = __builtin_amdgcn_udot4(x.z, 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(x.z, 0x01000100u, O, false);
        E = __builtin_amdgcn_udot4(x.w, 0x00010001u, E, false);
        O = __builtin_amdgcn_udot4(x.w, 0x01000100u, O, false);
    }
    return L ? fold64((uint64_t)E + ((uint64_t)O << 8)) : 0u;
}

// ---------------------------------------------------------------------------------------------
// Variable-length batches through LDS (inet_stream_kernel): a wave owns windows of 64 consecutive
// packets (interleaved over the grid). A window whose packets are packed (each starts where the
// previous one ends) and at least 16 B long is one contiguous span: it arrives in 6 KiB items by
// LDS-DMA into the wave's slot (rows only as far as the span reaches, the first and last at the
// default cache policy), and lane l sums the item's bytes [96 l, 96 l + 96) piece by piece into the
// packet they belong to (the window's packet starts in LDS; a 16-B piece holds at most one packet
// boundary): even- and odd-addressed bytes by v_dot4_u32_u8 running sums (the word sum is E + 256 O,
// the same residue as the dword sums), split at a boundary by the running sum before its dword
// plus that dword's bytes below it; each packet's part goes into its LDS accumulator once per lane
// (ds_add_u64). The
// next item's DMA (or the next packed window's first) is in flight while the current one is
// summed. Lane l finishes packet l (fold, odd-start swap, pseudo header). Other windows take one
// lane per packet when every packet is at most kShortMax bytes, else the flat chunk stream
// (flat_window), inside the same kernel. 16 waves per CU.
// ---------------------------------------------------------------------------------------------
constexpr int kStWaves = 16;
constexpr uint32_t kStSlot = 6144;
constexpr uint32_t kStLane = kStSlot / 64;   // 96 bytes of an item per lane
static_assert(kStLane % 16 == 0, "whole pieces per lane");

template <int MODE>
__global__ __launch_bounds__(kStWaves * 64, 1) void inet_stream_kernel(IParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t slots[kStWaves * kStSlot];
    __shared__ unsigned long long acc_s[kStWaves][64];
    __shared__ uint32_t start_s[kStWaves][64];
    __shared__ uint8_t mark_s[kStWaves][64], list_s[kStWaves][64];
    typedef __attribute__((address_space(3))) void lds_void;
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slot = slots + wave * kStSlot;
    unsigned long long *acc = acc_s[wave];
    uint32_t *st = start_s[wave];
    acc[lane] = 0ull;
    mark_s[wave][lane] = 0;
    const uint64_t n = p.n, nwin = (n + 63) >> 6, W = (uint64_t)gridDim.x * kStWaves;

    // A window's metadata (lane l: packet w0 + l) and, once it has arrived, its geometry.
    struct Meta {
        uint64_t off;
        uint32_t len;
    };
    struct Geo {
        bool packed;
        uint64_t a0;      // the span's first 16-B piece (byte address)
        uint32_t total;   // span bytes from a0 to its last byte (exclusive)
        uint32_t items;
    };
    auto meta = [&](uint64_t wi) -> Meta {
        const uint64_t i = wi * 64 + (uint64_t)lane;
        Meta m{0ull, 0u};
        if (wi < nwin && i < n) {
            m.off = p.off[i];
            m.len = p.len[i];
        }
        return m;
    };
    auto geo = [&](uint64_t wi, const Meta &m) -> Geo {
        Geo g{false, 0ull, 0u, 0u};
        if (wi >= nwin) return g;
        const bool act = wi * 64 + (uint64_t)lane < n;
        const uint64_t end = m.off + m.len;
        const uint64_t pend = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(end >> 32), 1) << 32) |
                              (uint32_t)__shfl_up((int)(uint32_t)end, 1);
        const bool ok = !act || (m.len >= 16 && (lane == 0 || m.off == pend));
        if (__ballot(!ok) != 0ull) return g;
        const uint64_t am = __ballot(act);
        const int last = 63 - __builtin_clzll(am);
        const uint64_t s0 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(m.off >> 32), 0) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)m.off, 0);
        const uint64_t e1 = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(end >> 32), last) << 32) |
                            (uint32_t)__shfl((int)(uint32_t)end, last);
        const uint64_t a0 = (p.base + s0) & ~15ull, tot = p.base + e1 - a0;
        if (tot >= (1ull << 31)) return g;
        g.packed = true;
        g.a0 = a0;
        g.total = (uint32_t)tot;
        g.items = (uint32_t)((tot + kStSlot - 1) / kStSlot);
        return g;
    };
    // item k of a packed window: pieces from a0 + k kStSlot up to the span's last byte's piece
    auto dma = [&](const Geo &g, uint32_t k) {
        const uint32_t base = k * kStSlot;
        const uint32_t span16 = (g.total + 15u) & ~15u;
        const uint32_t need = span16 - base < kStSlot ? span16 - base : kStSlot;
        const uint64_t a = g.a0 + base + 16ull * (uint32_t)lane;
        const uint32_t o = 16u * (uint32_t)lane;
        lds_void *la = (lds_void *)slot, *lb = (lds_void *)(slot + 4096);
        if (o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 0, 0);
        if (1024u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 1024, 2);
        if (2048u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 2048, 2);
        if (3072u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a), la, 16, 3072, 2);
        if (4096u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a + 4096), lb, 16, 0, 2);
        if (5120u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(a + 4096), lb, 16, 1024, 0);
    };

    uint64_t wi = (uint64_t)blockIdx.x * kStWaves + wave;
    Meta cm = meta(wi);
    Geo cg = geo(wi, cm);
    if (cg.packed) dma(cg, 0);   // the first window's first item
    while (wi < nwin) {          // wave-uniform
        const uint64_t wn = wi + W;
        const Meta nm = meta(wn);   // in flight while the current window is summed
        const uint64_t w0 = wi * 64;
        if (!cg.packed) {
            const bool act = w0 + (uint64_t)lane < n;
            if (__ballot(act && cm.len > kShortMax) == 0ull) {   // short packets: one lane each
                if (act) {
                    u32x4 v[kShortPieces];
                    const uint64_t start = p.base + cm.off;
                    if (cm.len) short_issue(start, cm.len, v);
                    const uint32_t s0 = short_sum(v, start, cm.len);
                    const uint32_t m = (start & 1) ? swap16(s0) : s0;
                    p.out[w0 + lane] = (uint16_t)~fold64((uint64_t)pseudo<MODE>(p, w0 + lane, cm.len) + m);
                }
            } else {
                flat_window<true, MODE>(p, w0, lane, acc, mark_s[wave], list_s[wave]);
            }
            const Geo ng = geo(wn, nm);
            if (ng.packed) dma(ng, 0);
            wi = wn;
            cm = nm;
            cg = ng;
            continue;
        }
        const bool act = w0 + (uint64_t)lane < n;
        const uint32_t my = act ? (uint32_t)(p.base + cm.off - cg.a0) : cg.total;   // packet start in the span
        st[lane] = my;
        wave_lds_sync();
        const uint32_t st0 = st[0];
        Geo ng{false, 0ull, 0u, 0u};
        for (uint32_t k = 0; k < cg.items; k++) {
            __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's slot has landed
            u32x4 v[kStLane / 16];
#pragma unroll
            for (int q = 0; q < (int)(kStLane / 16); q++)
                v[q] = *reinterpret_cast<const u32x4 *>(slot + kStLane * (uint32_t)lane + 16u * (uint32_t)q);
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next DMA
            if (k + 1 < cg.items) {
                dma(cg, k + 1);
            } else {   // the next window's metadata has landed with this item: its first item now
                ng = geo(wn, nm);
                if (ng.packed) dma(ng, 0);
            }
            // ---- this lane's 96 bytes: positions [P0, P0 + 96) of the span ----
            const uint32_t P0 = k * kStSlot + kStLane * (uint32_t)lane;
#ifdef INET_ST_NOSUM   // measurement-only: the pieces XORed into the lane's own packet (wrong sums)
            if (P0 < cg.total) {
                uint32_t xx = 0;
#pragma unroll
                for (int q = 0; q < (int)(kStLane / 16); q++) xx ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
                atomicAdd(&acc[lane], (unsigned long long)xx);
            }
            if (false) {
#else
            if (P0 < cg.total) {
#endif
                int cur = 0;   // the packet holding P0 (or the first one, before st0)
#pragma unroll
                for (int b = 32; b >= 1; b >>= 1)
                    if (st[cur + b] <= P0) cur += b;
                uint32_t nxt = cur + 1 < 64 ? st[cur + 1] : cg.total;
                // the current packet's part: even- and odd-addressed bytes (sum = E + 256 O)
                uint32_t E = 0, O = 0;
                auto flush = [&]() {
                    const uint32_t part = E + (O << 8);
                    if (part) atomicAdd(&acc[cur], (unsigned long long)part);
                    E = O = 0;
                    cur++;
                    nxt = cur + 1 < 64 ? st[cur + 1] : cg.total;
                };
#pragma unroll
                for (int q = 0; q < (int)(kStLane / 16); q++) {
                    const uint32_t Pq = P0 + 16u * (uint32_t)q;
                    if (Pq >= cg.total) break;
                    u32x4 x = v[q];
                    if (Pq < st0 || cg.total - Pq < 16u) {   // the span's first or last piece
                        const uint32_t lo = Pq < st0 ? st0 - Pq : 0u;
                        const uint32_t hi = cg.total - Pq < 16u ? cg.total - Pq : 16u;
                        const uint32_t keep = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
                        x.x &= byte_mask(keep, 0);
                        x.y &= byte_mask(keep, 1);
                        x.z &= byte_mask(keep, 2);
                        x.w &= byte_mask(keep, 3);
                    }
                    if (nxt <= Pq) flush();   // a packet starts exactly at this piece
                    // running sums over the piece's dwords
                    const uint32_t e0 = __builtin_amdgcn_udot4(x.x, 0x00010001u, 0u, false);
                    const uint32_t o0 = __builtin_amdgcn_udot4(x.x, 0x01000100u, 0u, false);
                    const uint32_t e1 = __builtin_amdgcn_udot4(x.y, 0x00010001u, e0, false);
                    const uint32_t o1 = __builtin_amdgcn_udot4(x.y, 0x01000100u, o0, false);
                    const uint32_t e2 = __builtin_amdgcn_udot4(x.z, 0x00010001u, e1, false);
                    const uint32_t o2 = __builtin_amdgcn_udot4(x.z, 0x01000100u, o1, false);
                    const uint32_t e3 = __builtin_amdgcn_udot4(x.w, 0x00010001u, e2, false);
                    const uint32_t o3 = __builtin_amdgcn_udot4(x.w, 0x01000100u, o2, false);
                    // the next packet starts inside the piece's span bytes (in dword b / 4 at byte b % 4);
                    // the last packet's `nxt` is the span end, never a start
                    const uint32_t b = nxt - Pq, hi = cg.total - Pq < 16u ? cg.total - Pq : 16u;
                    if (b < hi) {
                        const uint32_t db = b >> 2, lm = (1u << (8u * (b & 3u))) - 1u;
                        uint32_t eb = db == 0 ? 0u : (db == 1 ? e0 : (db == 2 ? e1 : e2));
                        uint32_t ob = db == 0 ? 0u : (db == 1 ? o0 : (db == 2 ? o1 : o2));
                        const uint32_t xd = db == 0 ? x.x : (db == 1 ? x.y : (db == 2 ? x.z : x.w));
                        eb = __builtin_amdgcn_udot4(xd, 0x00010001u & lm, eb, false);
                        ob = __builtin_amdgcn_udot4(xd, 0x01000100u & lm, ob, false);
                        E += eb;
                        O += ob;
                        flush();
                        E = e3 - eb;
                        O = o3 - ob;
                    } else {
                        E += e3;
                        O += o3;
                    }
                }
                const uint32_t part = E + (O << 8);
                if (part) atomicAdd(&acc[cur], (unsigned long long)part);
            }
        }
        // ---- packet w0 + lane: fold, odd-start swap, pseudo header and init, complement ----
        wave_lds_sync();
        if (act) {
            const uint32_t m0 = fold64(acc[lane]);
            const uint32_t m = ((p.base + cm.off) & 1) ? swap16(m0) : m0;   // odd start: P = swap16(fold(M))
            p.out[w0 + lane] = (uint16_t)~fold64((uint64_t)pseudo<MODE>(p, w0 + lane, cm.len) + m);
        }
        acc[lane] = 0ull;
        wi = wn;
        cm = nm;
        cg = ng;
    }
}

// ---------------------------------------------------------------------------------------------
// Fixed-stride batches through LDS (inet_dma_kernel): the FCS headline kernel's load form. A wave
// item is four consecutive packets; the 16-B pieces from the first packet's start to the fourth
// packet's end (at most 6 KiB: dma_ok) arrive in the wave's 6 KiB LDS slot by global_load_lds (six
// 1 KiB rows, non-temporal, each only as far as the item's bytes reach: nothing past the last
// packet is read). Quarter q of the wave sums packet q of the item from the slot (ds_read_b128 of
// the packet's aligned pieces, lane j pieces j, j + 16, ...; edge pieces masked as in accumulate),
// row_sum, fold, pseudo header; the next item's DMA is in flight meanwhile. Items come from the
// work dispenser in guided chunks of consecutive items; lane 0 of each quarter stores its packet's
// u16, four adjacent ones per item. 16 waves per CU.
// ---------------------------------------------------------------------------------------------
constexpr int kDmaWaves = 16;
constexpr uint32_t kDmaSlot = 6144;
#ifndef INET_EDGE_AUX   // cache policy of a slot's first and last rows (measurement-only override)
#define INET_EDGE_AUX 0
#endif
constexpr int kDmaRounds = 7;   // pieces per lane: a packet of at most 1532 B (dma_ok) touches <= 98 pieces

template <int MODE>
__global__ __launch_bounds__(kDmaWaves * 64, 1) void inet_dma_kernel(IParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDmaWaves * kDmaSlot];
    typedef __attribute__((address_space(3))) void lds_void;
    const uint32_t lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint8_t *slot = lds + wave * kDmaSlot;
    const uint64_t n = p.n, items = (n + 3) >> 2;
    // items from the work dispenser: guided chunks of consecutive items (as fcs_dma_kernel's; the
    // waves of the chip run at different speeds, a static interleave ends with the slowest)
    fcs::Dispenser D(p.ctr, items, (uint64_t)gridDim.x * kDmaWaves, (uint64_t)blockIdx.x * kDmaWaves + wave,
                     (int)lane, 100, 4, 64);
    constexpr uint64_t kEnd = fcs::Dispenser::kEnd;
    // slot source of item i: the 16-B piece holding its first byte; pieces up to its last byte
    auto src_of = [&](uint64_t i) { return (p.base + 4 * i * p.stride) & ~15ull; };
    auto dma = [&](uint64_t i) {
        const uint64_t a = src_of(i);
        const uint64_t last = (4 * i + 3 < n ? 4 * i + 3 : n - 1);
        const uint32_t need = (uint32_t)(((p.base + last * p.stride + p.flen + 15) & ~15ull) - a);
        const uint64_t g = a + 16ull * lane;
        const uint32_t o = 16u * lane;
        lds_void *la = (lds_void *)slot, *lb = (lds_void *)(slot + 4096);
        // the first and last rows hold the lines the neighbouring items share: default policy
        if (o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), la, 16, 0, INET_EDGE_AUX);
        if (1024u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), la, 16, 1024, 2);
        if (2048u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), la, 16, 2048, 2);
        if (3072u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), la, 16, 3072, 2);
        if (4096u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g + 4096), lb, 16, 0, 2);
        if (5120u + o < need) __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g + 4096), lb, 16, 1024, INET_EDGE_AUX);
    };
    // the pseudo-header addresses of a packet (lane j == 0 of its quarter), one item ahead
    auto addr_of = [&](uint64_t i, uint32_t &s, uint32_t &d) {
        const uint64_t f = 4 * i + q;
        s = d = 0;
        if (MODE != kIp && j == 0 && f < n) {
            s = p.addr[2 * f];
            d = p.addr[2 * f + 1];
        }
    };
    uint64_t it = D.first();
    if (it == kEnd) return;
    dma(it);
    uint32_t as, ad;
    addr_of(it, as, ad);
    while (it != kEnd) {   // wave-uniform
        const uint64_t f = 4 * it + q;
        const bool act = f < n;
        const uint64_t start = p.base + f * p.stride, c0 = start & ~15ull, end = start + p.flen;
        const uint32_t nch = act ? (uint32_t)((((end + 15) & ~15ull) - c0) >> 4) : 0u;
        const uint32_t so = (uint32_t)(c0 - src_of(it));   // the packet's first piece in the slot
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's slot has landed
        u32x4 v[kDmaRounds];
#pragma unroll
        for (int r = 0; r < kDmaRounds; r++) {
            const uint32_t c = j + kGroup * r;
            v[r] = c < nch ? *reinterpret_cast<const u32x4 *>(slot + so + 16u * c) : u32x4{0u, 0u, 0u, 0u};
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the slot is free for the next DMA
        const uint32_t cs = as, cd = ad;
        const uint64_t nx = D.next(it);
        if (nx != kEnd) {
            dma(nx);
            addr_of(nx, as, ad);
        }
        uint64_t acc = 0;
#pragma unroll
        for (int r = 0; r < kDmaRounds; r++) {
            const uint32_t c = j + kGroup * r;
            u32x4 x = v[r];
            if (c == 0 || c + 1 == nch) {   // edge pieces: keep bytes in [start, end)
                const uint64_t ca = c0 + 16ull * c;
                const uint32_t lo = start > ca ? (uint32_t)(start - ca) : 0u;
                const uint32_t hi = end - ca < 16 ? (uint32_t)(end - ca) : 16u;
                const uint32_t keep = ((1u << hi) - 1u) & ~((1u << lo) - 1u);
                x.x &= byte_mask(keep, 0);
                x.y &= byte_mask(keep, 1);
                x.z &= byte_mask(keep, 2);
                x.w &= byte_mask(keep, 3);
            }
            acc += (uint64_t)x.x + x.y;
            acc += (uint64_t)x.z + x.w;
        }
        const uint32_t s = fold64(row_sum(fold64(acc)));
        const uint32_t m = (start & 1) ? swap16(s) : s;
        const uint32_t ps = pseudo_sd<MODE>(cs, cd, p.flen);
        if (j == 0 && act) p.out[f] = (uint16_t)~fold64((uint64_t)ps + m);
        it = nx;
    }
}

// ---------------------------------------------------------------------------------------------
// Short fixed-stride packets (inet_short_kernel): one lane per packet of at most kShortMax bytes
// (the IP header ip_hton checksums, src/ip.c:79-80). Each lane loads the (at most five) 16-B pieces
// its packet touches, masks the first and last, sums the even- and odd-addressed bytes by
// v_dot4_u32_u8, folds, and 64 results leave as one 128-B store. Two packets per lane are in
// flight (the next one's loads issued before the current one is summed); a grid of persistent
// waves walks the batch. The one-packet-per-quarter-wave kernels spend 16 lanes on a 20-B header.
// ---------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kThreads) void inet_short_kernel(IParams p) {
    const uint64_t G = (uint64_t)gridDim.x * kThreads;
    const uint32_t L = p.flen;
    uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    u32x4 v[kShortPieces], w[kShortPieces];
    if (i < p.n && L) short_issue(p.base + i * p.stride, L, v);
    while (i < p.n) {
        const uint64_t nx = i + G;
        if (nx < p.n && L) short_issue(p.base + nx * p.stride, L, w);   // the next packet in flight
        const uint64_t start = p.base + i * p.stride;
        const uint32_t s = short_sum(v, start, L);
        const uint32_t m = (start & 1) ? swap16(s) : s;   // odd start: P = swap16(fold(M))
        p.out[i] = (uint16_t)~fold64((uint64_t)pseudo<MODE>(p, i, L) + m);
        i = nx;
#pragma unroll
        for (int q = 0; q < kShortPieces; q++) v[q] = w[q];
    }
}

// dma_ok: fixed packets whose four-packet items fit a slot with the 16-B rounding of both ends
// (so at most kDmaRounds * 16 pieces a packet), and that fill at least half of their stride (the
// slot also carries the gaps between packets).
static bool dma_ok(const IParams &p) {
    return p.flen >= 64 && p.stride <= 2048 && 2 * (uint64_t)p.flen >= p.stride &&
           3 * p.stride + p.flen + 30 <= kDmaSlot && p.flen + 30 <= 16u * kGroup * kDmaRounds;
}

// The one routing decision (launch_inet launches what it returns; the engine leases a work counter
// exactly when it returns kDma).
Route route_inet(bool var, const IParams &p, uint64_t flat_min, uint64_t dma_min) {
    if (!p.n) return Route::kNone;
    if (var && p.n > dma_min) return Route::kStream;
    if (!var && p.n > flat_min && p.flen <= kShortMax) return Route::kShort;   // lane per packet
    if (!var && p.n > dma_min && dma_ok(p)) return Route::kDma;
    if (p.n > flat_min) return Route::kFlat;
    return Route::kGroup;
}

hipError_t launch_inet(bool var, int mode, const IParams &p, int cus, uint64_t flat_min, uint64_t dma_min,
                       hipStream_t st) {
    (void)hipGetLastError();   // report this launch's own error, not an earlier call's
    const Route r = route_inet(var, p, flat_min, dma_min);
    if (r == Route::kNone) return hipSuccess;
    if (r == Route::kStream) {
        const uint64_t nwin = (p.n + 63) / 64;
        const uint64_t want = (nwin + kStWaves - 1) / kStWaves;
        const int grid = (int)(want < (uint64_t)cus ? want : (uint64_t)cus);
        if (mode == kTcp) hipLaunchKernelGGL((inet_stream_kernel<kTcp>), dim3(grid), dim3(kStWaves * 64), 0, st, p);
        else if (mode == kUdp) hipLaunchKernelGGL((inet_stream_kernel<kUdp>), dim3(grid), dim3(kStWaves * 64), 0, st, p);
        else hipLaunchKernelGGL((inet_stream_kernel<kIp>), dim3(grid), dim3(kStWaves * 64), 0, st, p);
        return hipGetLastError();
    }
    if (r == Route::kShort) {
        const uint64_t want = (p.n + kThreads - 1) / kThreads, cap = (uint64_t)cus * 8;
        const int grid = (int)(want < cap ? want : cap);
        if (mode == kTcp) hipLaunchKernelGGL((inet_short_kernel<kTcp>), dim3(grid), dim3(kThreads), 0, st, p);
        else if (mode == kUdp) hipLaunchKernelGGL((inet_short_kernel<kUdp>), dim3(grid), dim3(kThreads), 0, st, p);
        else hipLaunchKernelGGL((inet_short_kernel<kIp>), dim3(grid), dim3(kThreads), 0, st, p);
        return hipGetLastError();
    }
    if (r == Route::kDma) {
        if (!p.ctr) return hipErrorInvalidValue;
        const uint64_t items = (p.n + 3) / 4;
        const uint64_t want = (items + kDmaWaves - 1) / kDmaWaves;
        const int grid = (int)(want < (uint64_t)cus ? want : (uint64_t)cus);
        if (mode == kTcp) hipLaunchKernelGGL((inet_dma_kernel<kTcp>), dim3(grid), dim3(kDmaWaves * 64), 0, st, p);
        else if (mode == kUdp) hipLaunchKernelGGL((inet_dma_kernel<kUdp>), dim3(grid), dim3(kDmaWaves * 64), 0, st, p);
        else hipLaunchKernelGGL((inet_dma_kernel<kIp>), dim3(grid), dim3(kDmaWaves * 64), 0, st, p);
        return hipGetLastError();
    }
    if (r == Route::kFlat) {
        const uint64_t windows = (p.n + 63) / 64, per_block = kThreads / 64;
        const uint64_t want = (windows + per_block - 1) / per_block, cap = (uint64_t)cus * 8;
        const int grid = (int)(want < cap ? want : cap);
#define INET_FLAT(V, M) hipLaunchKernelGGL((inet_flat_kernel<V, M>), dim3(grid), dim3(kThreads), 0, st, p)
        if (var) {
            if (mode == kTcp) INET_FLAT(true, kTcp);
            else if (mode == kUdp) INET_FLAT(true, kUdp);
            else INET_FLAT(true, kIp);
        } else {
            if (mode == kTcp) INET_FLAT(false, kTcp);
            else if (mode == kUdp) INET_FLAT(false, kUdp);
            else INET_FLAT(false, kIp);
        }
#undef INET_FLAT
        return hipGetLastError();
    }
    const uint64_t per_block = kThreads / kGroup;   // Route::kGroup
    uint64_t want = (p.n + per_block - 1) / per_block;
    const uint64_t cap = (uint64_t)cus * 8;   // 32 waves per CU, persistent over the packets
    const int grid = (int)(want < cap ? want : cap);
#define INET_LAUNCH(V, M) hipLaunchKernelGGL((inet_kernel<V, M>), dim3(grid), dim3(kThreads), 0, st, p)
    if (var) {
        if (mode == kTcp) INET_LAUNCH(true, kTcp);
        else if (mode == kUdp) INET_LAUNCH(true, kUdp);
        else INET_LAUNCH(true, kIp);
    } else {
        if (mode == kTcp) INET_LAUNCH(false, kTcp);
        else if (mode == kUdp) INET_LAUNCH(false, kUdp);
        else INET_LAUNCH(false, kIp);
    }
#undef INET_LAUNCH
    return hipGetLastError();
}

}  // namespace inet
