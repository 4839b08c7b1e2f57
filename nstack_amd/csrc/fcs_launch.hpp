// fcs_launch.hpp — host-side launchers implemented in fcs_kernel.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fcs_tables.hpp"

namespace fcs {

struct KParams {
    uint64_t base;          // fixed: frame 0 start; var: arena start
    uint64_t stride;        // fixed only
    const uint64_t *off;    // var only
    const uint32_t *len;    // var only
    uint32_t *out;
    uint64_t n;             // frames
    uint64_t lo4, hi4;      // readable byte range, dword-rounded (never crosses a page)
    uint32_t flen;          // fixed: frame length
    uint32_t fseg;          // fixed: segments per frame
    uint32_t zmax;          // max leading zero bytes any front lane can see (mask loop bound)
    const uint32_t *blob;   // constant tables (kBlobWords)
    uint64_t *dbg;          // diagnostic stamp sink (FCS_STAMPS builds only; null otherwise)
    uint8_t *ok;            // verify mode: ok[i] = 1 iff frame i (FCS trailer included) checks
    unsigned long long *bad;//   ... and *bad += number of frames that do not (else both null)
    unsigned long long *ctr;// zeroed device work counter for a dynamic schedule (null: static interleave)
    // Arena-stream kernel (fcs_stream_kernel) and its follow-up: units of kStUnitFrames frames the
    // stream kernel did not take (not packed, or a length outside 64..1536) are appended to ulist
    // (count in *ucount, zeroed before the launch); fcs_flat_kernel with ulist set processes exactly
    // those units (and returns at once when there are none).
    uint32_t *ulist;
    uint32_t *ucount;
    uint32_t *listed_out;   // fcs_flat_kernel<listed units>: stores *ucount here (test introspection)
};
// Arena-stream kernel geometry: units of frames handed out by the dispenser; 64-B lane chunks at
// fixed arena positions, 64 per 4 KiB item; frames of 64..1536 B, packed within a unit.
#ifndef FCS_ST_UNIT   // measurement-only override
#define FCS_ST_UNIT 512
#endif
constexpr uint32_t kStUnitFrames = FCS_ST_UNIT;
constexpr uint32_t kStMinLen = 64, kStMaxLen = 1536;

// Workgroup sizes (one workgroup per CU either way: the LDS tables take 150 KiB). The 1504..1536-B
// single-segment kernel and frames of kWideSegs (3) or more segments run 8 waves per CU: 2 per SIMD
// beat 4 per SIMD by 1-7 % on 1518-B and 9000-B frames (tools/ab.py; 4, 6, 12 and
// 14 waves were slower or equal). The generic kernel on 1-2 segments (64..1500 B, 1540 B) loses
// 8-16 % at 8 waves and keeps 16 (3000 B: equal), as do the variable-length kernels (the flat
// kernel on IMIX: 4358 vs 3728 GB/s at 8 waves).
#ifndef FCS_WG_THREADS   // measurement-only overrides (tools/variants.sh)
#define FCS_WG_THREADS 1024
#endif
#ifndef FCS_FIXED_WG_THREADS
#define FCS_FIXED_WG_THREADS 512
#endif
constexpr int kWgThreads = FCS_WG_THREADS;             // variable-length kernels
constexpr int kFixedWgThreads = FCS_FIXED_WG_THREADS;  // fixed-length kernels
static_assert(kWgThreads % 64 == 0 && kWgThreads <= 1024, "workgroup = 1..16 waves (LDS scratch holds 16)");
static_assert(kFixedWgThreads % 64 == 0 && kFixedWgThreads <= 1024, "workgroup = 1..16 waves");
#ifndef FCS_WIDE_SEGS   // measurement-only override
#define FCS_WIDE_SEGS 3
#endif
constexpr uint32_t kWideSegs = FCS_WIDE_SEGS;   // fixed frames of >= 3 segments (> 3072 B): 8 waves per CU
constexpr uint32_t kSingleMaxLead = 32;    // fcs_single_kernel: <= 32 leading bytes to mask

// Single-frame kernel of the drop-in ether_fcs (fcs_one_kernel): the frame travels inside the
// kernel arguments, right-aligned in a 1536-byte window (zeros before it), one wave of 64 lanes
// takes 24 bytes each. Tables: the four slice-by-4 tables, then nibble tables of A_{24 * 2^k},
// k = 0..5, for the lane tree (kOneBlobWords words).
constexpr uint32_t kOneBytes = 1536;
constexpr uint32_t kOneBlobWords = 1024 + 6 * 128;
struct OneArgs {
    uint64_t *flag;          // device address of a mapped host word: (seq << 32) | FCS
    const uint32_t *blob;    // kOneBlobWords
    uint32_t seq;
    uint32_t kinit;          // A_len(0xFFFFFFFF): the all-ones start carried over the frame
    uint32_t data[kOneBytes / 4];
};

// Small TX (or RX verify) batches in mapped host memory (fcs_tx_small_kernel): 1..kTxSmallMax
// frames of up to kOneBytes bytes each, their offsets, lengths and A_len(0xFFFFFFFF) in the kernel
// arguments. One workgroup per frame writes its FCS (TX: out[i]) or its check (RX: ok[i]) into
// library-owned mapped memory, never into the caller's frames, so a kernel left in flight by a
// failed call cannot write into an arena the caller has reused (the host stores the FCSs after the
// completion). The last frame done (device counter `count`, which has reached count_base when the
// launch starts) stores `seq` into `flag`.
// The same kernel body with the frame list in (mapped) memory instead of the arguments, for any
// batch size (fcs_small_list_kernel): RX batches checked while the next recvmmsg runs.
struct ListArgs {
    uint64_t *flag;
    const uint32_t *blob;    // kOneBlobWords
    const uint32_t *kinit;   // A_L(0xFFFFFFFF), L = 0 .. kOneBytes (device memory)
    uint8_t *base;           // device address of the (mapped) arena
    const uint64_t *off;     // device addresses of mapped arrays of n entries
    const uint32_t *len;
    uint8_t *ok;             // null: TX (out[i] = FCS); else RX verify
    uint32_t *out;
    unsigned long long *count;
    uint64_t count_base;
    uint64_t seq;
    uint32_t n, pad;
};
constexpr uint32_t kTxSmallMax = 64;
struct TxSmallArgs {
    uint64_t *flag;
    const uint32_t *blob;    // kOneBlobWords
    uint8_t *base;           // device address of the (mapped) arena
    uint8_t *ok;             // null: TX (out[i] = FCS, mapped); else RX verify: ok[i] (mapped) per frame
    uint32_t *out;
    unsigned long long *count;
    uint64_t count_base;
    uint64_t seq;
    uint32_t n, pad;
    uint64_t off[kTxSmallMax];
    uint32_t len[kTxSmallMax];
    uint32_t kinit[kTxSmallMax];
};


// Fixed length: the launcher's kernel choice, shared with the host's grid sizing.
inline bool fixed_tiny(const KParams &p) { return p.hi4 - p.lo4 < 2 * (uint64_t)kChunkBytes; }
inline bool fixed_single(const KParams &p) {
#ifdef FCS_NO_SINGLE   // measurement-only build
    return false;
#else
    return p.fseg == 1 && p.zmax <= kSingleMaxLead;
#endif
}
// Windowed variable-length batches (and the short fixed-length route) take fcs_flat_kernel.
// LDS-DMA kernel (fcs_dma_kernel): one-segment frames of kDmaMinLen..kDmaCover bytes whose four
// consecutive frames (one wave item) fit one 6 KiB slot: the slot starts at floor16 of the first
// frame's start and must reach ceil4 of the fourth frame's end (3 stride + len <= 6144 - 15 - 3),
// and the arena must hold a whole slot (the last items' slots are clamped to its end).
#ifndef FCS_DMA_WG_THREADS   // measurement-only override
#define FCS_DMA_WG_THREADS 1024
#endif
constexpr int kDmaWgThreads = FCS_DMA_WG_THREADS;  // one 6 KiB LDS slot per wave
static_assert(kDmaWgThreads % 64 == 0 && kDmaWgThreads <= 1024, "LDS holds 16 slots next to the 64 KiB tables");
// Batches of at least this many items (4 frames) per wave of the grid hand their tail out
// dynamically (KParams::ctr): below it the static share alone balances well enough.
constexpr uint64_t kDmaDynMinItemsPerWave = 16;
inline bool fixed_dma(const KParams &p) {
#ifdef FCS_NO_DMA   // measurement-only build
    return false;
#else
    return p.fseg == 1 && p.flen >= kDmaMinLen && p.flen <= kDmaCover && p.stride <= 2048 &&
           3 * p.stride + p.flen <= kDmaItemBytes - 18 && p.hi4 - p.lo4 >= 2 * kDmaItemBytes;
#endif
}
// Frame-interleaved segment kernel (fcs_segil_kernel): fixed lengths over kDmaCover bytes, any
// stride; units of 4 frames, 12 waves per workgroup (8 KiB LDS slots). A frame costs
// m = ceil(len / 1524) items whatever its front segment holds; the register-load generic kernel
// walks ceil(len / 1536) segments. The segment kernel is selected (tools/ab.py, one process per
// length, round 3) when
//   - m >= 4 (4573 B and 6100 B equal, 9000 B +3 to +8.5 %, 65536 B +16 %), or
//   - m = 3 and the generic kernel needs 3 segments too, i.e. len > 3072 (3100 B +17 %,
//     3300 B +16 %; 3049 B -4 %: the generic kernel covers it in 2 segments), or m = 3 and a wider
//     segment width covers the frame in two items (round 5: 3049-3072 B on WD 26, +8.5 to +10.6 %
//     against the generic kernel), or
//   - m = 2 and len >= 1950 (2000 B +2.7 %, 2285 B +7.4 %; 1560-1900 B -1 to -4 %, and 1525-1536 B
//     are a single generic segment: -26 %).
// Segment width for a batch fixed_segil() takes: 24 (fcs_segil_kernel, 1524-B segments) or another
// width with lane tables (fcs_segw_kernel<WD>, segments of wide_cover(WD): 15..23 for 900..1412 B,
// 26 / 30 / 32 for 1604 / 1860 / 1988 B): the least per-lane work per frame, m (WD + kSegItemWords)
// for m = ceil(len / cover) items of WD words each plus a fixed per-item cost in word equivalents
// (merge, lane shift, row XOR, waits, four run issues); ties keep the earlier candidate.
#ifndef FCS_SEG_ITEM_WORDS   // measurement-only override of the per-item cost
#define FCS_SEG_ITEM_WORDS 8
#endif
constexpr uint32_t kSegItemWords = FCS_SEG_ITEM_WORDS;
__host__ __device__ constexpr int segment_wd(uint32_t len) {
#ifdef FCS_SEGW_FORCE   // measurement-only: one width for every segment batch
    return (void)len, FCS_SEGW_FORCE;
#else
    int best = 24;
    uint64_t cost = (uint64_t)((len + kDmaCover - 1) / kDmaCover) * (24u + kSegItemWords);
    // the bank-safe widths with lane tables (wide_mid_ok: 15..23), then the wide kernel's three
    const int wds[10] = {15, 16, 18, 19, 20, 22, 23, 26, 30, 32};
    for (int i = 0; i < 10; i++) {
        const uint64_t m = (len + wide_cover(wds[i]) - 1) / wide_cover(wds[i]);
        if (m * ((uint64_t)wds[i] + kSegItemWords) < cost) {
            cost = m * ((uint64_t)wds[i] + kSegItemWords);
            best = wds[i];
        }
    }
    return best;
#endif
}
constexpr uint32_t kSegilMinLen2 = 1950;
constexpr int kSegilWgThreads = 768;
inline bool fixed_segil(const KParams &p) {
#ifdef FCS_NO_SEGIL   // measurement-only build
    (void)p;
    return false;
#else
    const uint64_t m = (p.flen + kDmaCover - 1) / kDmaCover;
    if (p.flen <= kDmaCover || fixed_tiny(p)) return false;
#ifdef FCS_SEGIL_ANY   // measurement-only: every fixed length over 1524 B
    return true;
#endif
    if (m >= 4) return true;
    // 3049..3072 B: two generic segments, unless a wider segment width covers the frame in two items
    if (m == 3) return p.flen > 2u * (uint32_t)kSegBytes || segment_wd(p.flen) != 24;
    return p.flen >= kSegilMinLen2;
#endif
}
// Wide LDS-DMA kernel (fcs_wide_kernel): one-item frames of kWideMinLen..kWideCover bytes (128-B
// lane windows, 12 waves, 8 KiB slots) whose four consecutive frames fit one slot, as fixed_dma().
// Against the kernels these lengths took before (tools/ab.py, one process): 1537 B
// +22 %, 1600-1949 B +24 to +27 % (generic kernel, two segments), 1950-1988 B +23 to +26 %
// (segment kernel). The 104-B windows (WD 26) then took 1537-1604 B another +26 to +27 % (13 waves
// instead of 12), and 120-B windows (WD 30) 1605-1787 B +16 to +19 %. Round 4 (one process per
// length): WD 26 also takes 1525-1536 B (+15 to +17 % against the single-segment kernel; the 128-B
// windows had lost there) and 1477-1495 B, between the mid band and the LDS-DMA kernel (+7 %
// against the flat kernel).
#ifndef FCS_WIDE_MIN   // measurement-only override of the band's lower end
#define FCS_WIDE_MIN 1525
#endif
constexpr uint32_t kWideMinLen = FCS_WIDE_MIN;
__host__ __device__ constexpr int wide_threads(int wd) { return wd == 32 ? 768 : (wd > 24 ? 832 : 1024); }   // 12 / 13 / 16 waves
// Mid-length band (round 4): fixed lengths kWideMidMinLen..wide_cover(kWideMidMax) (870..1476 B)
// take the narrowest bank-safe width whose 16 windows cover the frame (wide_mid_ok), 6 KiB slots,
// 16 waves, instead of the flat kernel. tools/ab.py, one process per length, with the one-AND front
// masks: 870 B +5.8 %, 880 B +3.9 %, 900 B +5.7 %, 965 B +4.4 %, 1000 B +1.8 %,
// 1093 B +7.1 %, 1157 B +10.5 %, 1300 B +7.7 %; below the band 837 B -2.3 %, 860 B -1.0 %, and
// WD 14 at 720 B -9 %.
#ifndef FCS_WIDE_MID_MIN   // measurement-only override of the band's lower end (0: no mid band)
#define FCS_WIDE_MID_MIN 870
#endif
constexpr uint32_t kWideMidMinLen = FCS_WIDE_MID_MIN;
__host__ __device__ constexpr int wide_mid_wd(uint32_t len) {
    for (int wd = kWideMidMin; wd <= kWideMidMax; wd++)
        if (wide_mid_ok(wd) && wide_cover(wd) >= len) return wd;
    return 0;
}
// Window dwords for a fixed batch: 26 (104-B windows) or 30 (120-B windows), 7 KiB slots and 13
// waves, when the frame and its item fit those, else 32 (128-B windows, 8 KiB slots, 12 waves);
// 0: not the wide kernel.
inline int wide_wd(const KParams &p) {
#ifdef FCS_NO_WIDE   // measurement-only build
    (void)p;
    return 0;
#else
    if (kWideMidMinLen && p.flen >= kWideMidMinLen && p.flen <= wide_cover(kWideMidMax)) {
        const int wd = wide_mid_wd(p.flen);
        return (p.stride <= 2048 && 3 * p.stride + p.flen <= wide_slot(wd) - 18 &&
                p.hi4 - p.lo4 >= 2 * (uint64_t)wide_slot(wd)) ? wd : 0;
    }
    // 1477..1495 B: above the mid band, below the LDS-DMA kernel
#ifdef FCS_WIDE_NO_PRE   // measurement-only: those on the flat kernel
    const bool pre = false;
#else
    const bool pre = p.flen > wide_cover(kWideMidMax) && p.flen < kDmaMinLen;
#endif
    if ((p.flen < kWideMinLen && !pre) || p.stride > 4096) return 0;
#ifndef FCS_WIDE_NO26   // measurement-only: the 128-B windows for the whole band
    if (p.flen <= kWideCover26 && 3 * p.stride + p.flen <= wide_slot(26) - 18 &&
        p.hi4 - p.lo4 >= 2 * (uint64_t)wide_slot(26))
        return 26;
#endif
#ifndef FCS_WIDE_NO30   // measurement-only: no 120-B windows
    if (p.flen <= kWideCover30 && 3 * p.stride + p.flen <= wide_slot(30) - 18 &&
        p.hi4 - p.lo4 >= 2 * (uint64_t)wide_slot(30))
        return 30;
#endif
    if (p.flen <= kWideCover && 3 * p.stride + p.flen <= wide_slot(32) - 18 && p.hi4 - p.lo4 >= 2 * (uint64_t)wide_slot(32))
        return 32;
    return 0;
#endif
}
inline bool fixed_wide(const KParams &p) { return wide_wd(p) != 0; }
// Eight-lane groups (fcs_wide_kernel<WD, 8>): fixed lengths kWide8MinLen..wide8_cover(28) bytes,
// eight frames per item, the narrowest bank-safe WD (11..28) whose eight windows cover the frame,
// when the item's eight frames fit the width's slot.
#ifndef FCS_WIDE8_MIN   // measurement-only override of the band's lower end (0: no eight-lane groups)
#define FCS_WIDE8_MIN 400
#endif
constexpr uint32_t kWide8MinLen = FCS_WIDE8_MIN;
// The windows' LDS reads: the most live lanes of one 32-lane half on one dword bank (every window
// word shifts all lanes' banks alike, so word 0 stands for all). Four frames share a half; strides
// that put them on the same bank phase (e.g. 512 or 768 B) give 4-way conflicts, which measured
// slower than the flat kernel (512 B -4.6 %, 768 B -3.6 %; 741 B, 3-way, -1.6 %).
inline int wide_bank_load(const KParams &p, int wd, uint32_t G) {
    const uint32_t step = wide_step(wd);
    const uint32_t cf = (p.flen - 1u) / step < G - 1u ? (p.flen - 1u) / step : G - 1u;
    int worst = 0;
    for (int half = 0; half < 2; half++) {
        int cnt[32] = {0};
        for (int l = 32 * half; l < 32 * half + 32; l++) {
            const uint32_t c = (uint32_t)l % G, g = (uint32_t)l / G;
            if (c > cf) continue;
            const uint64_t x = p.base + g * p.stride + p.flen - step * c - wide_win(wd);
            const int b = (int)((x >> 2) & 31u);
            if (++cnt[b] > worst) worst = cnt[b];
        }
    }
    return worst;
}
inline int wide8_wd(const KParams &p) {
    if (!kWide8MinLen || p.flen < kWide8MinLen || p.flen > wide8_cover(28) || p.stride > 2048) return 0;
    int wd = kWide8Min;
    while (!wide8_ok(wd) || wide8_cover(wd) < p.flen) wd++;
    return (7 * p.stride + p.flen <= wide_slot(wd) - 18 && p.hi4 - p.lo4 >= 2 * (uint64_t)wide_slot(wd) &&
            wide_bank_load(p, wd, 8) <= 2) ? wd : 0;
}
inline bool fixed_wide8(const KParams &p) { return wide8_wd(p) != 0; }
// Four-lane groups (fcs_wide_kernel<WD, 4>): fixed lengths kWide4MinLen..kWide8MinLen - 1, sixteen
// frames per item, the narrowest width (9..26, not 17) whose four windows cover the frame, when the
// item's sixteen frames fit the width's slot and the 32-lane halves' bank load is at most 2.
#ifndef FCS_WIDE4_MIN   // measurement-only override of the band's lower end (0: no four-lane groups)
#define FCS_WIDE4_MIN 130
#endif
constexpr uint32_t kWide4MinLen = FCS_WIDE4_MIN;
inline int wide4_wd(const KParams &p) {
    if (!kWide4MinLen || p.flen < kWide4MinLen || p.flen > wide4_cover(kWide4Max) || p.stride > 2048 ||
        (kWide8MinLen && p.flen >= kWide8MinLen))
        return 0;
    int wd = kWide4Min;
    while (!wide4_ok(wd) || wide4_cover(wd) < p.flen) wd++;
    return (15 * p.stride + p.flen <= wide_slot(wd) - 18 && p.hi4 - p.lo4 >= 2 * (uint64_t)wide_slot(wd) &&
            wide_bank_load(p, wd, 4) <= 2) ? wd : 0;
}
inline bool fixed_wide4(const KParams &p) { return wide4_wd(p) != 0; }
// Short-frame kernel (fcs_short_kernel<W>): fixed lengths of 1..kShortMaxLen bytes, one lane per
// frame, the W-dword window ending at the frame end loaded into registers (any stride). Against the
// flat chunk stream (tools/ab.py, one process per length): 60 B +11.5 %, 64 B
// +10.4 %, 32 B +10.2 %, 66..74 B +6.0 to +6.7 %, 80..96 B +1.7 to +3.6 % (W = 16 and 24 with the
// loads one item ahead), 100 B +27 %, 128 B +1.6 to +10 %.
#ifndef FCS_SHORT_MAX   // measurement-only override (0: no short-frame kernel)
#define FCS_SHORT_MAX 128
#endif
constexpr uint32_t kShortMaxLen = FCS_SHORT_MAX;
__host__ __device__ constexpr int short_wd(uint32_t len) { return len <= 64 ? 16 : (len <= 96 ? 24 : (len <= 128 ? 32 : 0)); }
static_assert(short_wd(1) == 16 && short_wd(65) == 24 && short_wd(97) == 32 && short_wd(129) == 0, "short-frame widths");
inline bool fixed_short(const KParams &p) {
    return p.flen >= 1 && p.flen <= kShortMaxLen && short_wd(p.flen) != 0 && !fixed_tiny(p);
}
// Fixed-length batches of frames up to this length (and more than the small-batch threshold) take
// the flat chunk stream when no slot kernel takes them: a 64-B frame then costs one lane instead of a
// quarter-wave. Measured against the quarter-wave kernel (tools/ab.py): 64 B 11x,
// 576 B 2.1x, 1300 B +6.5 %; 1504..1536 B stay on the single kernel (the flat kernel is 9 % slower
// at 1518 B). The slot kernels go first where their slots take the batch.
#ifndef FCS_FIXED_FLAT_MAX   // measurement-only override (0 = never)
#define FCS_FIXED_FLAT_MAX 1503
#endif
constexpr uint32_t kFixedFlatMaxLen = FCS_FIXED_FLAT_MAX;
// The flat kernel hands its 64-frame windows out dynamically once there are at least this many
// windows per wave of the grid; the generic and segment kernels their 4-frame units from this many
// units per wave (the LDS-DMA family: kDmaDynMinItemsPerWave items).
#ifndef FCS_FLAT_DYN_MIN   // measurement-only override (a huge value keeps the flat kernel static)
#define FCS_FLAT_DYN_MIN 4
#endif
constexpr uint64_t kFlatDynMinWindowsPerWave = FCS_FLAT_DYN_MIN;
#ifndef FCS_FIXED_DYN_MIN   // measurement-only override (a huge value keeps the kernel static)
#define FCS_FIXED_DYN_MIN 4
#endif
constexpr uint64_t kFixedDynMinUnitsPerWave = FCS_FIXED_DYN_MIN;
#ifndef FCS_SHORT_WG_PER_CU   // measurement-only: workgroups per CU (2: -6 to -8 %)
#define FCS_SHORT_WG_PER_CU 1
#endif

// THE routing decision for fixed-length batches: launch_fixed (engine) sizes the
// grid and leases the work counter from it, launch_fixed_route (fcs_kernel.hip) launches exactly
// the kernel it names, and fcs_debug_fixed_route names it. big: more frames than the small-batch
// threshold (fcs_engine_set_var_threshold).
enum class FixedKernel : uint8_t { kShort, kFlat, kWide4, kWide8, kWide16, kSegment, kDma, kTiny, kSingle, kGeneric };
struct FixedRoute {
    FixedKernel kernel;
    int wd;                  // short: window dwords W; wide: WD; LDS-DMA: front mask words; tiny: 1 if single
    bool tiny;               // flat / generic: the tiny-arena instantiation (guarded loads)
    int threads;             // workgroup size
    uint32_t item_frames;    // frames per dispenser item (unit, window)
    uint64_t dyn_min;        // items per wave from which the schedule is dynamic (0: always static)
    uint32_t zmax;           // the front-mask bound the kernel is launched with
};
inline FixedRoute route_fixed(const KParams &p, bool big) {
    const bool tiny = fixed_tiny(p);
    const bool slot = !tiny && (fixed_wide4(p) || fixed_wide8(p) || fixed_wide(p) || fixed_dma(p));
    if (big && fixed_short(p))
        return {FixedKernel::kShort, short_wd(p.flen), false, kWgThreads, 64, kDmaDynMinItemsPerWave, p.zmax};
    if (p.flen <= kFixedFlatMaxLen && big && !slot)   // len == null tells the flat kernel the length is p.flen
        return {FixedKernel::kFlat, 0, tiny, kWgThreads, 64, kFlatDynMinWindowsPerWave, kChunkBytes};
    if (!tiny && fixed_wide4(p)) {
        const int wd = wide4_wd(p);
        return {FixedKernel::kWide4, wd, false, wide_threads(wd), 16, kDmaDynMinItemsPerWave, p.zmax};
    }
    if (!tiny && fixed_wide8(p)) {
        const int wd = wide8_wd(p);
        return {FixedKernel::kWide8, wd, false, wide_threads(wd), 8, kDmaDynMinItemsPerWave, p.zmax};
    }
    if (!tiny && fixed_wide(p)) {
        const int wd = wide_wd(p);
        return {FixedKernel::kWide16, wd, false, wide_threads(wd), 4, kDmaDynMinItemsPerWave, p.zmax};
    }
    if (fixed_segil(p))
        return {FixedKernel::kSegment, segment_wd(p.flen), false, kSegilWgThreads, 4, kFixedDynMinUnitsPerWave, p.zmax};
    if (!tiny && fixed_dma(p)) {   // the front lane masks kDmaCover - len bytes, lanes 3/7/11 one word
        const uint32_t z = kDmaCover - p.flen > 4 ? kDmaCover - p.flen : 4;
        return {FixedKernel::kDma, z <= 8 ? 2 : (int)(kSingleMaxLead / 4), false, kDmaWgThreads, 4, kDmaDynMinItemsPerWave, z};
    }
    if (tiny) return {FixedKernel::kTiny, fixed_single(p) ? 1 : 0, true, kWgThreads, 4, 0, p.zmax};   // wd: single
    if (fixed_single(p)) return {FixedKernel::kSingle, 0, false, kFixedWgThreads, 4, 0, p.zmax};
    return {FixedKernel::kGeneric, 0, false, p.fseg >= kWideSegs ? kFixedWgThreads : kWgThreads, 4,
            kFixedDynMinUnitsPerWave, p.zmax};
}

hipError_t launch_fcs(bool var, bool windowed, const KParams &p, int grid, hipStream_t st);
// Launches the kernel route_fixed(p, big) named as `r` (p.zmax = r.zmax) and records it for
// last_fixed_launch.
hipError_t launch_fixed_route(const FixedRoute &r, const KParams &p, int grid, hipStream_t st);
// The kernel the last launch_fixed_route call launched (test introspection): its route with
// threads/item fields as launched. Zero-initialised before any.
FixedRoute last_fixed_launch();
hipError_t launch_signal(uint64_t *flag, uint64_t v, hipStream_t st);
// Test-only: a one-lane kernel that waits for a nonzero mapped host word or `ticks` of the 100 MHz
// constant clock, whichever comes first (fcs_debug_hold_small).
hipError_t launch_hold(const uint32_t *word, uint64_t ticks, hipStream_t st);
hipError_t launch_one(const OneArgs &a, hipStream_t st);
hipError_t launch_tx_small(const TxSmallArgs &a, hipStream_t st);
hipError_t launch_small_list(const ListArgs &a, hipStream_t st);
hipError_t launch_fill(void *p, uint64_t bytes, uint64_t seed, uint64_t off, hipStream_t st);
hipError_t launch_read_stream(const void *p, uint64_t bytes, uint32_t *sink, hipStream_t st);
hipError_t launch_dma_stream(const KParams &p, int grid, hipStream_t st);
// load_only: fcs_stream_kernel<true>, the measurement form behind fcs_stream_load_dev
hipError_t launch_stream(const KParams &p, int grid, hipStream_t st, bool load_only = false);
hipError_t launch_short(const KParams &p, int grid, hipStream_t st);
hipError_t launch_tx_store(uint8_t *base, uint64_t stride, const uint32_t *len, const uint32_t *crc,
                           uint64_t n, hipStream_t st);

}  // namespace fcs
