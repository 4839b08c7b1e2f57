// fcs_tables.hpp — host-side construction of the constant tables the FCS kernel keeps in LDS.
//
// The CRC in src/ether_fcs.c:4-19 is CRC-32/ISO-HDLC: a reflected LFSR over GF(2) with
// polynomial 0xEDB88320 whose register starts and ends complemented. Writing A_n for the
// linear operator "advance the register over n zero bytes", appending one 4-byte word w is
// s' = A_4(s ^ w), and that is what the slice-by-4 tables T3..T0 evaluate. Everything the
// kernel needs beyond that is an A_n (or its inverse) for a handful of n, tabulated by nibble:
//   lane tables   L_j = A_{96 j}         j = 0..15   (shift lane j's chunk to the frame end)
//   segment shift J   = A_{1536}                     (a lane's register accumulated over
//                                                     segment k is advanced by one segment
//                                                     before segment k+1's value is XORed in)
//   chain combine H48 = A_48, H24 = A_24             (a lane runs its 24 words as four
//                                                     independent 6-word chains and merges
//                                                     them as a tree: A_48(A_24(a)^b) ^
//                                                     (A_24(c)^d))
//   front init    INV[z] = A_z^{-1}(0xFFFFFFFF)      (register value that, after z leading
//                                                     zero bytes, equals the all-ones init)
//   M   = A_{-768}                                   (unused since round 3: the half-unit
//                                                     kernel that needed it is gone; kept so the
//                                                     blob and LDS offsets below stay put)
//   chunk shifts  C_c = A_{96 c}         c = 0..15   (flat variable-length kernel: a lane's
//                                                     chunk index is data-dependent, so the
//                                                     table is indexed by c, not by lane)
//   (and the LDS-DMA, arena-stream and wide kernels' tables, listed at their blob offsets below)
// These are constants of the algorithm, computed once per process. (Frame bytes are checksummed
// on the host only by fcs_host_crc.cpp, the error path's slice-by-16, not from these tables.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <vector>

namespace fcs {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr int kChunkBytes = 96;                       // bytes per lane per segment
constexpr int kChunkWords = kChunkBytes / 4;          // 24
constexpr int kGroup = 16;                            // lanes per frame (quarter wave)
constexpr int kSegBytes = kChunkBytes * kGroup;       // 1536
constexpr int kJumpBytes = kSegBytes;                 // 1536 (segment accumulation)

// LDS layout of the kernel (bytes). Data tables: T_k[b], replica r (= lane & 31) lives at
//   half(k)*65536 + b*256 + odd(k)*128 + r*4    with T3,T2 in half 0 and T1,T0 in half 1,
// so the address is one v_perm of {x.byte_k, lane constant} and every ds_read_b32 of a
// 32-lane group hits 32 distinct banks. Lane tables are stored per lane & 31 (bank = lane) with
// the content of lane & 15, so two frames in one 32-lane group never conflict.
constexpr uint32_t kLdsData = 0;        // 131072 B
constexpr uint32_t kLdsLane = 131072;   // 8 nibble tables x 16 entries x 32 slots x 4 B = 16384
constexpr uint32_t kLdsJump = 147456;   // 8 x 16 x 4 B = 512 (A_1536)
constexpr uint32_t kLdsH48 = 147968;    // 8 x 16 x 4 B = 512 (A_48)
constexpr uint32_t kLdsH24 = 148480;    // 8 x 16 x 4 B = 512 (A_24)
constexpr uint32_t kLdsInv = 148992;    // 96 x 4 B = 384
constexpr uint32_t kLdsM768 = 149376;   // 8 x 16 x 4 B = 512 (A_{-768})
constexpr uint32_t kLdsWave = 149888;   // per-wave scratch for the variable-length kernel
constexpr uint32_t kLdsWaveBytes = 256; //   (four 64-entry frame lists per wave)
constexpr uint32_t kLdsBad = kLdsWave + 16 * kLdsWaveBytes;    // 153984: per-wave u64 failing-frame count (verify)
constexpr uint32_t kLdsBytes = kLdsBad + 16 * 8;                // 154112
// The flat variable-length kernel keeps C_c in the lane-table region instead (it never uses the
// per-lane tables): nibble table t of C_c at kLdsFlat + c*kFlatStride + t*64 + e*4. The stride is
// 136 dwords (== 8 mod 64 banks), so lanes with different c spread over the banks: 2.09 cycles per
// 32-lane access on IMIX items against 2.45 at 132 dwords and 3.96 at 128 (bank simulation with
// random nibbles). Per-wave frame-start marks and rank -> lane lists follow it.
constexpr uint32_t kLdsFlat = kLdsLane;
constexpr uint32_t kFlatStride = 544;
constexpr uint32_t kFlatBytes = 16 * kFlatStride;              // 8704
constexpr uint32_t kLdsFlatMark = kLdsFlat + kFlatBytes;        // 16 waves x 64 B
constexpr uint32_t kLdsFlatList = kLdsFlatMark + 16 * 64;       // 16 waves x 64 B
static_assert(kLdsFlatList + 16 * 64 <= kLdsJump, "flat scratch fits the lane-table region");

// LDS-DMA fixed kernel (fcs_dma_kernel): frames arrive in LDS by global_load_lds, and lane c of a
// frame's 16 reads its 96-byte window [E - e_c - 96, E - e_c) from there (E = frame end). Chunks
// are 96 B except c = 3, 7, 11 (92 B: the window's first word belongs to lane c + 1 and is
// masked), so e_c = 96 c - 4 (c / 4) and the 16 windows start on 16 distinct LDS banks
// (e_c / 4 mod 32 = 8 (c mod 4) - c / 4): the data reads of one frame never conflict, where
// 96-B steps put four lanes on each bank. 16 lanes cover e_15 + 96 = 1524 bytes.
__host__ __device__ constexpr uint32_t dma_end_off(int c) { return 96u * (uint32_t)c - 4u * (uint32_t)(c >> 2); }
__host__ __device__ constexpr bool dma_short_lane(int c) { return (c & 3) == 3 && c < 15; }
constexpr uint32_t kDmaCover = dma_end_off(15) + kChunkBytes;   // 1524
constexpr uint32_t kDmaMinLen = 1496;                            // front lane masks <= 28 B
constexpr uint32_t kDmaItemBytes = 6144;                         // one wave's LDS slot: 6 x 1 KiB DMA
// Wide LDS-DMA kernel (fcs_wide_kernel, fixed lengths just over kDmaCover): 128-byte lane windows
// ending e_c = 124 c before the frame end. Each window's first word is its neighbour's last (masked
// in every lane but the frame's front lane), and the 16 windows start on 16 distinct banks
// ((e_c / 4) mod 32 = -c mod 32). 16 lanes cover e_15 + 128 = 1988 bytes; four frames per 8 KiB slot.
// Narrower widths where four frames fit a 7 KiB slot (13 waves): 104-byte windows every 100 B
// (cover 1604 B, banks 25 c mod 32) and 120-byte windows every 116 B (cover 1860 B, banks 29 c mod
// 32). Template parameter WD = window dwords (26, 30 or 32).
constexpr uint32_t kWideWin = 128;                               // the widest window (INV table size)
__host__ __device__ constexpr uint32_t wide_win(int wd) { return 4u * (uint32_t)wd; }
__host__ __device__ constexpr uint32_t wide_step(int wd) { return 4u * (uint32_t)wd - 4u; }
__host__ __device__ constexpr uint32_t wide_cover(int wd) { return 15u * wide_step(wd) + wide_win(wd); }
__host__ __device__ constexpr uint32_t wide_slot(int wd) { return wd == 32 ? 8192u : (wd > 24 ? 7168u : 6144u); }
// Mid-length windows (round 4): WD = kWideMidMin..kWideMidMax dwords (cover 900..1476 B), 6 KiB
// slots (four frames), 16 waves. Only widths whose 16 window starts fall on 16 distinct dword banks
// are used: (WD - 1) c mod 32 must differ for c = 0..15, so WD - 1 must not be a multiple of 4 (WD 17
// and 21 are skipped). Narrower widths (below 870 B) measured no faster than the flat kernel
// (DESIGN.md §3.2d).
#ifndef FCS_WIDE_MID_WD_MIN   // the narrowest mid-length width (11..14: measurement builds)
#define FCS_WIDE_MID_WD_MIN 15
#endif
constexpr int kWideMidMin = FCS_WIDE_MID_WD_MIN, kWideMidMax = 24;
static_assert(kWideMidMin >= 11 && kWideMidMin <= 20, "mid-length widths the launch switch instantiates");
__host__ __device__ constexpr bool wide_mid_ok(int wd) { return wd >= kWideMidMin && wd <= kWideMidMax && (wd - 1) % 4 != 0; }
// Eight-lane groups (round 4): eight frames per wave item, eight windows per frame, the bank-safe
// WD = 11 .. 28 dwords (cover 32 WD - 28 = 324 .. 868 B); 6 KiB slots up to WD 24, 7 KiB (13 waves)
// above.
constexpr int kWide8Min = 11, kWide8Max = 28;
__host__ __device__ constexpr uint32_t wide8_cover(int wd) { return 7u * wide_step(wd) + wide_win(wd); }
__host__ __device__ constexpr bool wide8_ok(int wd) { return wd >= kWide8Min && wd <= kWide8Max && (wd - 1) % 4 != 0; }
// Four-lane groups (round 4): sixteen frames per wave item, four windows per frame, WD = 9 .. 26
// (cover 16 WD - 12 = 132 .. 404 B), WD 17 skipped (windows 0 and 2 on one bank).
constexpr int kWide4Min = 9, kWide4Max = 26;
__host__ __device__ constexpr uint32_t wide4_cover(int wd) { return 3u * wide_step(wd) + wide_win(wd); }
__host__ __device__ constexpr bool wide4_ok(int wd) { return wd >= kWide4Min && wd <= kWide4Max && (wd - 1) % 16 != 0; }
constexpr uint32_t kWideCover = wide_cover(32);                  // 1988
constexpr uint32_t kWideCover26 = wide_cover(26);                // 1604
constexpr uint32_t kWideCover30 = wide_cover(30);                // 1860

// Global "blob" the kernel copies into LDS at start; words kBlobLane.. are in LDS order.
constexpr uint32_t kBlobSlice = 0;                      // uint32 [4][256]   (T0..T3)
constexpr uint32_t kBlobLane = 1024;                    // uint32 [8][16][32]
constexpr uint32_t kBlobJump = kBlobLane + 8 * 16 * 32; // uint32 [8][16]
constexpr uint32_t kBlobH48 = kBlobJump + 8 * 16;       // uint32 [8][16]
constexpr uint32_t kBlobH24 = kBlobH48 + 8 * 16;        // uint32 [8][16]
constexpr uint32_t kBlobInv = kBlobH24 + 8 * 16;        // uint32 [96]
constexpr uint32_t kBlobM768 = kBlobInv + kChunkBytes;  // uint32 [8][16]
constexpr uint32_t kBlobFlat = kBlobM768 + 8 * 16;      // uint32 [16][136] (C_c, LDS order)
constexpr uint32_t kBlobLaneDma = kBlobFlat + kFlatBytes / 4;   // uint32 [8][16][32]: A_{e_c}
constexpr uint32_t kBlobMerge = kBlobLaneDma + 8 * 16 * 32;     // uint32 [11][8][16]: A_{8k}, k = 1..11
// Arena-stream variable-length kernel (fcs_stream_kernel): chunk shifts A_{64 j} (j = 0..23),
// word shifts A_{4 i} (i = 0..16), inverse byte shifts A_{-d} (d = 1..4), each a nibble table
// [8][16], and K1[sigma] = A_{64 - sigma}(0xFFFFFFFF) (sigma = 0..63).
constexpr int kStChunkTabs = 24, kStWordTabs = 17, kStInvTabs = 4;
constexpr uint32_t kBlobStream = kBlobMerge + 11 * 8 * 16;
constexpr uint32_t kBlobStreamK1 = kBlobStream + (kStChunkTabs + kStWordTabs + kStInvTabs) * 128;
// Wide LDS-DMA kernel: lane tables A_{124 c} (WD 32) and A_{100 c} (WD 26) in the LDS-DMA layout
// [8][16][32], INV[z] for z < 128.
constexpr uint32_t kBlobLaneWide = kBlobStreamK1 + 64;
constexpr uint32_t kBlobLaneWide26 = kBlobLaneWide + 8 * 16 * 32;
constexpr uint32_t kBlobLaneWide30 = kBlobLaneWide26 + 8 * 16 * 32;   // A_{116 c} (WD 30)
constexpr uint32_t kBlobInvWide = kBlobLaneWide30 + 8 * 16 * 32;
// Mid-length wide kernels: lane tables A_{(4 WD - 4) c} for WD = kWideMidMin..kWideMidMax in the
// LDS-DMA layout [8][16][32] (one set per width, unused widths included so the offsets stay simple).
constexpr uint32_t kBlobLaneMid = kBlobInvWide + kWideWin;
// Eight-lane groups: lane tables A_{(4 WD - 4) (slot mod 8)} for WD = kWide8Min..kWide8Max (one set
// per width, unused widths included).
constexpr uint32_t kBlobLane8 = kBlobLaneMid + (kWideMidMax - kWideMidMin + 1) * 8 * 16 * 32;
constexpr uint32_t kBlobLane4 = kBlobLane8 + (kWide8Max - kWide8Min + 1) * 8 * 16 * 32;   // (slot mod 4)
constexpr uint32_t kBlobWords = kBlobLane4 + (kWide4Max - kWide4Min + 1) * 8 * 16 * 32;
static_assert((kLdsInv - kLdsLane) / 4 == kBlobInv - kBlobLane, "blob/LDS order");
static_assert((kLdsM768 - kLdsLane) / 4 == kBlobM768 - kBlobLane, "blob/LDS order");

struct Tables {
    uint32_t T[4][256];
    uint8_t top_inv[256];   // index i with (T0[i] >> 24) == byte (unique for a CRC table)

    Tables() {
        for (uint32_t b = 0; b < 256; b++) {
            uint32_t r = b;
            for (int i = 0; i < 8; i++) r = (r >> 1) ^ ((r & 1u) ? kPoly : 0u);
            T[0][b] = r;
        }
        for (int k = 1; k < 4; k++)
            for (int b = 0; b < 256; b++)
                T[k][b] = (T[k - 1][b] >> 8) ^ T[0][T[k - 1][b] & 0xFF];
        for (int b = 0; b < 256; b++) top_inv[T[0][b] >> 24] = (uint8_t)b;
    }
    // A_1: one zero byte.
    uint32_t zstep(uint32_t s) const { return (s >> 8) ^ T[0][s & 0xFF]; }
    // A_1^{-1}: s = (p >> 8) ^ T0[p & 0xFF]; the top byte of s names p & 0xFF.
    uint32_t zunstep(uint32_t s) const {
        uint32_t i = top_inv[s >> 24];
        return ((s ^ T[0][i]) << 8) | i;
    }
    uint32_t shift(uint32_t s, long n) const {
        for (; n > 0; n--) s = zstep(s);
        for (; n < 0; n++) s = zunstep(s);
        return s;
    }
    // Nibble table of A_n: entry [t][e] = A_n(e << 4t). A_n is linear: the images of the 32 bits.
    void nibble_table(long n, uint32_t out[8][16]) const {
        uint32_t img[32];
        for (int b = 0; b < 32; b++) img[b] = shift(1u << b, n);
        for (int t = 0; t < 8; t++)
            for (int e = 0; e < 16; e++) {
                uint32_t v = 0;
                for (int b = 0; b < 4; b++)
                    if (e >> b & 1) v ^= img[4 * t + b];
                out[t][e] = v;
            }
    }
    std::vector<uint32_t> blob() const {
        std::vector<uint32_t> b(kBlobWords, 0u);
        for (int k = 0; k < 4; k++) std::memcpy(&b[kBlobSlice + 256 * k], T[k], 1024);
        uint32_t nt[8][16];
        for (int slot = 0; slot < 32; slot++) {
            nibble_table((long)kChunkBytes * (slot % kGroup), nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobLane + (t * 16 + e) * 32 + slot] = nt[t][e];
        }
        nibble_table(kJumpBytes, nt);
        for (int t = 0; t < 8; t++)
            for (int e = 0; e < 16; e++) b[kBlobJump + t * 16 + e] = nt[t][e];
        nibble_table(48, nt);
        for (int t = 0; t < 8; t++)
            for (int e = 0; e < 16; e++) b[kBlobH48 + t * 16 + e] = nt[t][e];
        nibble_table(24, nt);
        for (int t = 0; t < 8; t++)
            for (int e = 0; e < 16; e++) b[kBlobH24 + t * 16 + e] = nt[t][e];
        for (int z = 0; z < kChunkBytes; z++) b[kBlobInv + z] = shift(0xFFFFFFFFu, -(long)z);
        nibble_table(-768, nt);
        for (int t = 0; t < 8; t++)
            for (int e = 0; e < 16; e++) b[kBlobM768 + t * 16 + e] = nt[t][e];
        for (int c = 0; c < 16; c++) {
            nibble_table((long)kChunkBytes * c, nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobFlat + c * (kFlatStride / 4) + t * 16 + e] = nt[t][e];
        }
        for (int slot = 0; slot < 32; slot++) {
            nibble_table((long)dma_end_off(slot % kGroup), nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobLaneDma + (t * 16 + e) * 32 + slot] = nt[t][e];
        }
        for (int k = 1; k <= 11; k++) {   // chain-merge shifts of the LDS-DMA kernel
            nibble_table(8L * k, nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobMerge + (k - 1) * 128 + t * 16 + e] = nt[t][e];
        }
        // arena-stream kernel: A_{64 j}, A_{4 i}, A_{-d}, K1
        int q = 0;
        auto put = [&](long n) {
            nibble_table(n, nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobStream + q * 128 + t * 16 + e] = nt[t][e];
            q++;
        };
        for (int j = 0; j < kStChunkTabs; j++) put(64L * j);
        for (int i = 0; i < kStWordTabs; i++) put(4L * i);
        for (int d = 1; d <= kStInvTabs; d++) put(-(long)d);
        for (int sg = 0; sg < 64; sg++) b[kBlobStreamK1 + sg] = shift(0xFFFFFFFFu, 64 - sg);
        for (int slot = 0; slot < 32; slot++) {   // wide kernel, both widths
            nibble_table((long)wide_step(32) * (slot % kGroup), nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobLaneWide + (t * 16 + e) * 32 + slot] = nt[t][e];
            nibble_table((long)wide_step(26) * (slot % kGroup), nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobLaneWide26 + (t * 16 + e) * 32 + slot] = nt[t][e];
            nibble_table((long)wide_step(30) * (slot % kGroup), nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[kBlobLaneWide30 + (t * 16 + e) * 32 + slot] = nt[t][e];
        }
        for (int z = 0; z < (int)kWideWin; z++) b[kBlobInvWide + z] = shift(0xFFFFFFFFu, -(long)z);
        for (int wd = kWideMidMin; wd <= kWideMidMax; wd++)   // mid-length wide kernels
            for (int slot = 0; slot < 32; slot++) {
                nibble_table((long)wide_step(wd) * (slot % kGroup), nt);
                for (int t = 0; t < 8; t++)
                    for (int e = 0; e < 16; e++)
                        b[kBlobLaneMid + (wd - kWideMidMin) * 4096 + (t * 16 + e) * 32 + slot] = nt[t][e];
            }
        for (int wd = kWide8Min; wd <= kWide8Max; wd++)   // eight-lane groups
            for (int slot = 0; slot < 32; slot++) {
                nibble_table((long)wide_step(wd) * (slot % 8), nt);
                for (int t = 0; t < 8; t++)
                    for (int e = 0; e < 16; e++) b[kBlobLane8 + (wd - kWide8Min) * 4096 + (t * 16 + e) * 32 + slot] = nt[t][e];
            }
        for (int wd = kWide4Min; wd <= kWide4Max; wd++)   // four-lane groups
            for (int slot = 0; slot < 32; slot++) {
                nibble_table((long)wide_step(wd) * (slot % 4), nt);
                for (int t = 0; t < 8; t++)
                    for (int e = 0; e < 16; e++) b[kBlobLane4 + (wd - kWide4Min) * 4096 + (t * 16 + e) * 32 + slot] = nt[t][e];
            }
        return b;
    }
    // Tables of the single-frame kernel (fcs_launch.hpp OneArgs): T0..T3, then A_{24 * 2^k}.
    std::vector<uint32_t> one_blob() const {
        std::vector<uint32_t> b(1024 + 6 * 128, 0u);
        for (int k = 0; k < 4; k++) std::memcpy(&b[256 * k], T[k], 1024);
        uint32_t nt[8][16];
        for (int k = 0; k < 6; k++) {
            nibble_table(24L << k, nt);
            for (int t = 0; t < 8; t++)
                for (int e = 0; e < 16; e++) b[1024 + k * 128 + t * 16 + e] = nt[t][e];
        }
        return b;
    }
};

}  // namespace fcs
