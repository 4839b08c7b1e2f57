// fcs_kernel.hip — batched Ethernet FCS (CRC-32/ISO-HDLC) for CDNA4 / gfx950 (MI355X).
//
// Replaces the per-frame byte loop of ether_fcs() (/root/reference/src/ether_fcs.c:13-16) with
// one launch over many independent frames. Result per frame is bit-identical to ether_fcs().
//
// Work decomposition:
//   * one HALF-WAVE (32 lanes) per frame; lane j owns the 48-byte chunk that ends 48*j bytes
//     before the frame end, so a 32-lane group covers one 1536-byte "segment"; longer frames
//     are walked segment by segment, front to back (jumbo 9000 B = 6 segments);
//   * each lane loads its chunk with 3 x global_load_dwordx4 + 1 dword from a 4-byte aligned
//     address (measured: this layout streams HBM at the same rate as a fully coalesced read),
//     re-aligns it to the frame end with v_alignbyte_b32 and zeroes bytes before the frame start;
//   * the lane runs a slice-by-4 CRC over its 12 words: 4 ds_read_b32 per word from byte tables
//     replicated 32x in LDS (replica = lane & 31 -> every 32-lane LDS access is bank-conflict
//     free), addressed by a single v_perm_b32 per lookup;
//   * the frame's initial all-ones register is injected as the front lane's start value
//     INV[z] = A_z^{-1}(~0) (z = zero bytes in front of the frame start), so no length-dependent
//     constant is needed; across segments a lane's register jumps over the other lanes' bytes
//     with J = A_1488;
//   * at the frame end lane j shifts its register by 48*j zero bytes (per-lane nibble tables,
//     bank = lane), the 32 registers are XOR-reduced with DPP, and lane 31 stores ~crc.
// No MFMA: this is a byte-stream codec bounded by HBM read bandwidth (roofline: DESIGN.md §4).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fcs_tables.hpp"
#include "fcs_launch.hpp"

namespace fcs {

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kHalvesPerWg = kWgThreads / 32;   // 16 waves; LDS (145 KiB) admits one WG per CU



struct Item {
    uint64_t end;   // byte address one past the frame's last byte
    uint32_t len;
    uint32_t m;     // segments
};

// Loads through address space 1 (global): flat loads would also count on lgkmcnt and make every
// LDS wait drain the prefetched chunk loads.
template <typename T>
__device__ __forceinline__ T gload(uint64_t addr) {
    return *reinterpret_cast<const __attribute__((address_space(1))) T *>(addr);
}

__device__ __forceinline__ uint32_t lds_rd(const uint8_t *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(lds + byte_addr);
}

// One 4-byte step: A_4(x) = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3].
// base0 = r*4 (half 0: T3 at +0, T2 at +128), base1 = 0x10000 | r*4 (half 1: T1, T0).
__device__ __forceinline__ uint32_t step4(const uint8_t *lds, uint32_t x, uint32_t base0,
                                          uint32_t base1) {
    const uint32_t a0 = __builtin_amdgcn_perm(x, base0, 0x0C020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(x, base0, 0x0C020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(x, base1, 0x0C020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(x, base1, 0x0C020700u);
    const uint32_t t3 = lds_rd(lds, a0);
    const uint32_t t2 = lds_rd(lds, a1 + 128);
    const uint32_t t1 = lds_rd(lds, a2);
    const uint32_t t0 = lds_rd(lds, a3 + 128);
    return t3 ^ t2 ^ t1 ^ t0;
}

// A_{48 j}(s): lane j's own nibble tables (entry e of table t at kLdsLane + t*2048 + e*128 + j*4).
__device__ __forceinline__ uint32_t lane_shift(const uint8_t *lds, uint32_t s, uint32_t lanebase) {
    uint32_t r = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 7) ? (s >> (4 * t - 7)) : (s << (7 - 4 * t));
        r ^= lds_rd(lds, ((sh & 0x780u) | lanebase) + t * 2048);
    }
    return r;
}

// A_1488(s): one shared table set (entry e of table t at kLdsJump + t*64 + e*4).
__device__ __forceinline__ uint32_t jump(const uint8_t *lds, uint32_t s) {
    uint32_t r = 0;
#pragma unroll
    for (int t = 0; t < 8; t++) {
        const uint32_t sh = (4 * t >= 2) ? (s >> (4 * t - 2)) : (s << 2);
        r ^= lds_rd(lds, ((sh & 0x3Cu) | kLdsJump) + t * 64);
    }
    return r;
}

// XOR over the 32 lanes of each half wave; the full value lands in lanes 16..31 / 48..63.
__device__ __forceinline__ uint32_t half_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast15 -> rows 1,3
    return v;
}

template <bool VAR>
__device__ __forceinline__ Item frame_item(const KParams &p, uint64_t f) {
    Item it;
    if (VAR) {
        const uint32_t L = p.len[f];
        it.end = p.base + p.off[f] + L;
        it.len = L;
        it.m = L ? (L + (kSegBytes - 1)) / kSegBytes : 1u;
    } else {
        it.end = p.base + f * p.stride + p.flen;
        it.len = p.flen;
        it.m = p.fseg;
    }
    return it;
}

// Raw loads of one lane chunk (issued early, consumed one item later) and what is needed to
// interpret them. Loads are unconditional and always inside [lo4, hi4): lanes with nothing to load
// read lo4, and a window that starts before lo4 (front lane of a frame at the very start of the
// arena) is clamped per 16-byte group and repaired after the data has landed (fixup_edge).
struct Chunk {
    u32x4a4 x0, x1, x2;
    uint32_t x3;
    int zr;          // bytes from chunk start to frame start (segment 0), -1 inside, 48 = no data
    uint32_t r;      // chunk start & 3 (realignment)
    int delta0;      // dwords group 0 was shifted by the low clamp (0 = not clamped)
    int delta1, delta2;
};

__device__ __forceinline__ uint64_t clamp64(uint64_t x, uint64_t lo, uint64_t hi) {
    return x < lo ? lo : (x > hi ? hi : x);
}

template <bool TINY>
__device__ __forceinline__ void issue_chunk(const KParams &p, const Item &it, uint32_t k, int j,
                                            bool act, Chunk &c) {
    const int64_t cend = (int64_t)it.end - (int64_t)kSegBytes * (int64_t)(it.m - 1 - k) -
                         (int64_t)kChunkBytes * j;
    const int64_t cstart = cend - kChunkBytes;
    const int64_t z = (k == 0) ? ((int64_t)(it.end - it.len) - cstart) : -1;
    c.zr = z < -1 ? -1 : (z > kChunkBytes ? kChunkBytes : (int)z);
    c.r = (uint32_t)cstart & 3u;
    const bool need = act && c.zr < kChunkBytes;
    const uint64_t a = need ? ((uint64_t)cstart & ~3ull) : p.lo4;
    if (TINY) {
        // Arena shorter than 64 B (host-selected variant): per-dword guarded loads.
        uint32_t d[13];
#pragma unroll
        for (int q = 0; q < 13; q++) {
            const uint64_t ad = a + 4 * q;
            d[q] = (need && ad >= p.lo4 && ad + 4 <= p.hi4) ? gload<uint32_t>(ad) : 0u;
        }
        c.x0 = u32x4a4{d[0], d[1], d[2], d[3]};
        c.x1 = u32x4a4{d[4], d[5], d[6], d[7]};
        c.x2 = u32x4a4{d[8], d[9], d[10], d[11]};
        c.x3 = d[12];
        c.delta0 = c.delta1 = c.delta2 = 0;
        return;
    }
    const uint64_t lo = p.lo4, hi16 = p.hi4 - 16, hi4 = p.hi4 - 4;
    const uint64_t g0 = clamp64(a, lo, hi16), g1 = clamp64(a + 16, lo, hi16), g2 = clamp64(a + 32, lo, hi16);
    c.delta0 = (int)((g0 - a) >> 2);
    c.delta1 = (int)((g1 - (a + 16)) >> 2);
    c.delta2 = (int)((g2 - (a + 32)) >> 2);
    c.x0 = gload<u32x4a4>(g0);
    c.x1 = gload<u32x4a4>(g1);
    c.x2 = gload<u32x4a4>(g2);
    c.x3 = gload<uint32_t>(clamp64(a + 48, lo, hi4));
}

// Undo the low clamp of one 16-byte group: true dword q = loaded dword q - delta (q >= delta);
// dwords q < delta lie before the arena start, hence before the frame start, and get masked.
__device__ __forceinline__ void unshift_group(uint32_t *g, int delta) {
    const uint32_t a = g[0], b = g[1], c = g[2], d = g[3];
    g[1] = delta == 1 ? a : (delta >= 2 ? a : b);
    g[2] = delta == 1 ? b : (delta == 2 ? a : (delta >= 3 ? a : c));
    g[3] = delta == 1 ? c : (delta == 2 ? b : (delta == 3 ? a : (delta >= 4 ? a : d)));
}

template <bool VAR, bool TINY>
struct Lane {
    const KParams &p;
    const uint8_t *lds;
    int j;
    uint32_t base0, base1, lanebase;
    uint64_t H;

    struct Pos {
        uint64_t f;
        uint32_t k;
        bool act;
        Item it;
    };

    __device__ __forceinline__ Pos next(const Pos &c) const {
        Pos n = c;
        n.k = c.k + 1;
        if (n.k >= c.it.m) {
            n.f = c.f + H;
            n.k = 0;
        }
        n.act = c.act && n.f < p.n;
        if (n.act && n.k == 0) n.it = frame_item<VAR>(p, n.f);
        return n;
    }

    // Consume one chunk: realign, mask, run the slice-by-4 chain, finish the frame if last.
    __device__ __forceinline__ void process(const Pos &c, const Chunk &ch, uint32_t &s) const {
        uint32_t d[13] = {ch.x0.x, ch.x0.y, ch.x0.z, ch.x0.w, ch.x1.x, ch.x1.y, ch.x1.z,
                          ch.x1.w, ch.x2.x, ch.x2.y, ch.x2.z, ch.x2.w, ch.x3};
        if (__any(ch.delta0 | ch.delta1 | ch.delta2)) {   // arena start only; wave-uniform branch
            unshift_group(d + 0, ch.delta0);
            unshift_group(d + 4, ch.delta1);
            unshift_group(d + 8, ch.delta2);
        }
        uint32_t w[12];
#pragma unroll
        for (int i = 0; i < 12; i++) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], ch.r);
        uint32_t x0;
        if (c.k == 0) {
#pragma unroll
            for (int i = 0; i < 12; i++) {
                if (4 * i < (int)p.zmax) {   // uniform bound: skip words no front lane can mask
                    int t = ch.zr - 4 * i;
                    t = t < 0 ? 0 : (t > 4 ? 4 : t);
                    w[i] &= (uint32_t)(0xFFFFFFFFull << (8 * t));
                }
            }
            const int zi = ch.zr < 0 ? 0 : (ch.zr > 47 ? 47 : ch.zr);
            const uint32_t iv = lds_rd(lds, kLdsInv + 4u * (uint32_t)zi);
            x0 = (ch.zr >= 0 && ch.zr < kChunkBytes) ? iv : 0u;
        } else {
            x0 = jump(lds, s);
        }
        uint32_t st = x0;
#pragma unroll
        for (int i = 0; i < 12; i++) st = step4(lds, st ^ w[i], base0, base1);
        s = st;

        const bool last = c.act && (c.k + 1 == c.it.m);
        if (__any(last)) {
            uint32_t v = last ? lane_shift(lds, s, lanebase) : 0u;
            v = half_xor(v);
            if (last && j == 31) p.out[c.f] = c.it.len ? ~v : 0u;
        }
    }
};

template <bool VAR, bool TINY>
__global__ __launch_bounds__(kWgThreads, 1) void fcs_kernel(KParams p) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];

    // ---- stage the tables into LDS (once per workgroup; the grid is persistent) ----
    {
        const int tid = threadIdx.x;
        // data: 8192 x 16 B; each b128 store = 4 replicas of one entry
        for (int i = tid; i < 8192; i += kWgThreads) {
            const int h = i >> 12;            // 64 KiB half
            const int b = (i >> 4) & 255;     // entry
            const int odd = (i >> 3) & 1;     // +128 slot
            // half 0: T3 (+0), T2 (+128); half 1: T1 (+0), T0 (+128)
            const int k = h == 0 ? (odd ? 2 : 3) : (odd ? 0 : 1);
            const uint32_t v = p.blob[kBlobSlice + 256 * k + b];
            u32x4 vv = {v, v, v, v};
            *reinterpret_cast<u32x4 *>(lds + kLdsData + (uint32_t)i * 16) = vv;
        }
        const uint32_t *src = p.blob + kBlobLane;
        uint32_t *dst = reinterpret_cast<uint32_t *>(lds + kLdsLane);
        for (int i = tid; i < (int)(kBlobInv + 48 - kBlobLane); i += kWgThreads) dst[i] = src[i];
        __syncthreads();
    }

    const int lane = threadIdx.x & 63;
    const int j = lane & 31;
    Lane<VAR, TINY> L{p, lds, j, (uint32_t)j * 4u, 0x10000u | ((uint32_t)j * 4u), kLdsLane | ((uint32_t)j * 4u),
                (uint64_t)gridDim.x * kHalvesPerWg};

    typename Lane<VAR, TINY>::Pos A, B;
    A.f = ((uint64_t)blockIdx.x * kHalvesPerWg) + (threadIdx.x >> 5);
    A.k = 0;
    A.act = A.f < p.n;
    A.it = A.act ? frame_item<VAR>(p, A.f) : Item{0, 0, 1};
    Chunk CA, CB;
    issue_chunk<TINY>(p, A.it, A.k, j, A.act, CA);
    uint32_t s = 0;

    // Two items in flight per lane: process one while the other's loads are outstanding.
    while (__any(A.act)) {
        B = L.next(A);
        issue_chunk<TINY>(p, B.it, B.k, j, B.act, CB);
        L.process(A, CA, s);
        if (!__any(B.act)) break;
        A = L.next(B);
        issue_chunk<TINY>(p, A.it, A.k, j, A.act, CA);
        L.process(B, CB, s);
    }
}

// Counter-based byte generator: 8-byte word q of the stream = splitmix64(seed + q).
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(256) void fill_splitmix_kernel(uint8_t *p, uint64_t bytes,
                                                            uint64_t seed, uint64_t off) {
    // Aligned body: 8-byte words of the stream that fall fully inside [off, off+bytes).
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
    for (; i + 3 * st < n16; i += 4 * st) {
        const u32x4 a = p[i], b = p[i + st], c = p[i + 2 * st], e = p[i + 3 * st];
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ e.x ^ e.y ^
               e.z ^ e.w;
    }
    for (; i < n16; i += st) {
        const u32x4 a = p[i];
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;   // keep the loads live; practically never stores
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
hipError_t launch_fcs(bool var, const KParams &p, int grid, hipStream_t st) {
    const bool tiny = p.hi4 - p.lo4 < 64;
    if (var && tiny)
        hipLaunchKernelGGL((fcs_kernel<true, true>), dim3(grid), dim3(kWgThreads), 0, st, p);
    else if (var)
        hipLaunchKernelGGL((fcs_kernel<true, false>), dim3(grid), dim3(kWgThreads), 0, st, p);
    else if (tiny)
        hipLaunchKernelGGL((fcs_kernel<false, true>), dim3(grid), dim3(kWgThreads), 0, st, p);
    else
        hipLaunchKernelGGL((fcs_kernel<false, false>), dim3(grid), dim3(kWgThreads), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_fill(void *p, uint64_t bytes, uint64_t seed, uint64_t off, hipStream_t st) {
    uint64_t words = bytes / 8 + 1;
    int grid = (int)((words + 255) / 256);
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(fill_splitmix_kernel, dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, seed, off);
    return hipGetLastError();
}

hipError_t launch_read_stream(const void *p, uint64_t bytes, uint32_t *sink, hipStream_t st) {
    hipLaunchKernelGGL(read_stream_kernel, dim3(8192), dim3(256), 0, st, (const u32x4 *)p, bytes / 16, sink);
    return hipGetLastError();
}

hipError_t launch_tx_store(uint8_t *base, uint64_t stride, const uint32_t *len, const uint32_t *crc,
                           uint64_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(tx_store_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, base, stride, len, crc, n);
    return hipGetLastError();
}

}  // namespace fcs
