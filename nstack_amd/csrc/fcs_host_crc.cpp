// fcs_host_crc.cpp — the library's own host CRC-32 (fcs_host_crc.hpp): the failure answers of the
// drop-in and the host batch forms, and the TX queue's batches below its GPU minimum.
//
// Three forms, one result:
// - Carry-less folding (x86 PCLMULQDQ, chosen at run time when the CPU has it). CRC-32 is the
//   message polynomial times x^32 modulo P, so a 128-bit block A may be replaced by any block
//   congruent to A * x^D mod P that sits D bits later: with A = A_hi x^64 + A_lo, that is
//   A_hi * (x^(64+D) mod P) + A_lo * (x^D mod P), two 64x32-bit carry-less products. Four
//   accumulators fold 64 bytes per step (D = 512) and are then folded into one (D = 128); the
//   remaining block is, modulo P, a 16-byte message of its own, so one slice-by-16 step from a zero
//   register turns it into the CRC register, and the table loop finishes the tail.
// - The same folding four 128-bit lanes wide (VPCLMULQDQ on 512-bit registers, AVX-512 hosts such as
//   the MI355X boxes' EPYC 9005): four accumulators of 64 bytes fold 256 bytes per step (D = 2048),
//   are folded into one (D = 512), which then takes 64 bytes per step; its four lanes are folded
//   into one 128-bit block (D = 384, 256, 128 side by side) and the 128-bit form finishes.
// - Slice-by-16 tables: sixteen 256-entry tables, table k advancing a byte past k further zero
//   bytes, so one step folds 16 input bytes with 16 independent lookups.
// Everything is derived at run time from the polynomial 0x04C11DB7 (reflected 0xEDB88320, the
// operator the reference's nibble table folds, src/ether_fcs.c:7-10); the register starts at ~0
// and is complemented at the end, which is what the reference's complement-folded table computes
// ("123456789" -> 0xCBF43926). It is the product's own code, not the test oracle.
#include "fcs_host_crc.hpp"

#include <immintrin.h>

#include <cstdlib>
#include <cstring>

namespace fcs {
namespace {

struct Slice16 {
    uint32_t t[16][256];
    Slice16() {
        for (uint32_t b = 0; b < 256; b++) {
            uint32_t r = b;
            for (int i = 0; i < 8; i++) r = (r >> 1) ^ (0xEDB88320u & (0u - (r & 1u)));
            t[0][b] = r;
        }
        for (int k = 1; k < 16; k++)
            for (uint32_t b = 0; b < 256; b++) t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xFFu];
    }
};

const Slice16 &tables16() {
    static const Slice16 s;
    return s;
}

inline uint32_t le32(const uint8_t *p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;   // x86-64 and every host this library builds for are little-endian
}

// One slice-by-16 step: the register after 16 more bytes.
inline uint32_t step16(const Slice16 &s, const uint8_t *p, uint32_t c) {
    const uint32_t a = le32(p) ^ c, b = le32(p + 4), d = le32(p + 8), e = le32(p + 12);
    return s.t[15][a & 0xFF] ^ s.t[14][(a >> 8) & 0xFF] ^ s.t[13][(a >> 16) & 0xFF] ^ s.t[12][a >> 24] ^
           s.t[11][b & 0xFF] ^ s.t[10][(b >> 8) & 0xFF] ^ s.t[9][(b >> 16) & 0xFF] ^ s.t[8][b >> 24] ^
           s.t[7][d & 0xFF] ^ s.t[6][(d >> 8) & 0xFF] ^ s.t[5][(d >> 16) & 0xFF] ^ s.t[4][d >> 24] ^
           s.t[3][e & 0xFF] ^ s.t[2][(e >> 8) & 0xFF] ^ s.t[1][(e >> 16) & 0xFF] ^ s.t[0][e >> 24];
}

// The same for 8 and 4 bytes (tables 7..0 and 3..0): the tail after the 16-byte steps takes at most
// one of each and three single bytes.
inline uint32_t step8(const Slice16 &s, const uint8_t *p, uint32_t c) {
    const uint32_t a = le32(p) ^ c, b = le32(p + 4);
    return s.t[7][a & 0xFF] ^ s.t[6][(a >> 8) & 0xFF] ^ s.t[5][(a >> 16) & 0xFF] ^ s.t[4][a >> 24] ^
           s.t[3][b & 0xFF] ^ s.t[2][(b >> 8) & 0xFF] ^ s.t[1][(b >> 16) & 0xFF] ^ s.t[0][b >> 24];
}

inline uint32_t step4(const Slice16 &s, const uint8_t *p, uint32_t c) {
    const uint32_t a = le32(p) ^ c;
    return s.t[3][a & 0xFF] ^ s.t[2][(a >> 8) & 0xFF] ^ s.t[1][(a >> 16) & 0xFF] ^ s.t[0][a >> 24];
}

uint32_t tables_crc(const uint8_t *p, size_t n, uint32_t c) {
    const Slice16 &s = tables16();
    for (; n >= 16; n -= 16, p += 16) c = step16(s, p, c);
    if (n >= 8) c = step8(s, p, c), p += 8, n -= 8;
    if (n >= 4) c = step4(s, p, c), p += 4, n -= 4;
    while (n--) c = (c >> 8) ^ s.t[0][(c ^ *p++) & 0xFFu];
    return c;
}

// ---- carry-less folding ----
// A 128-bit little-endian load of message bytes holds the coefficient of x^(127-k) in bit k
// (bit-reflected), and so does a 64-bit half for x^(63-k). The carry-less product of two such
// halves puts the coefficient of x^(126-t) in bit t: one power short, so each constant carries an
// x^-1. Folding constant pair for distance D: low half multiplies A_hi, high half A_lo.
uint64_t xpow_mod(unsigned n) {   // x^n mod P, bit d = coefficient of x^d
    uint64_t v = 1;
    for (unsigned i = 0; i < n; i++) v = (v << 1) ^ ((v & 0x80000000u) ? 0x104C11DB7ull : 0);
    return v;
}

uint64_t reflect64(uint64_t v) {   // coefficient of x^d moves to bit 63 - d
    uint64_t r = 0;
    for (int d = 0; d < 32; d++)
        if ((v >> d) & 1) r |= 1ull << (63 - d);
    return r;
}

struct FoldK {
    alignas(16) uint64_t k2048[2], k512[2], k384[2], k256[2], k128[2];
    static void set(uint64_t *k, unsigned d) {   // the pair for distance d bits
        k[0] = reflect64(xpow_mod(64 + d - 1));
        k[1] = reflect64(xpow_mod(d - 1));
    }
    FoldK() {
        set(k2048, 2048);
        set(k512, 512);
        set(k384, 384);
        set(k256, 256);
        set(k128, 128);
    }
};

const FoldK &fold_k() {
    static const FoldK k;
    return k;
}

__attribute__((target("pclmul,sse4.1"))) inline __m128i fold(__m128i x, __m128i k) {
    return _mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11));
}

// The register after n >= 64 bytes from register c (not complemented); *used = bytes consumed
// (a multiple of 16); the caller finishes the rest with the tables.
// Blocks x0..x3 hold the message's bytes [i - 64, i) folded so far; the rest of fold_crc from there.
__attribute__((target("pclmul,sse4.1"))) uint32_t fold_crc_from(const uint8_t *p, size_t n, size_t i, __m128i x0,
                                                                __m128i x1, __m128i x2, __m128i x3, size_t *used) {
    const FoldK &K = fold_k();
    const __m128i k512 = _mm_load_si128((const __m128i *)K.k512), k128 = _mm_load_si128((const __m128i *)K.k128);
    for (; i + 64 <= n; i += 64) {
        x0 = _mm_xor_si128(fold(x0, k512), _mm_loadu_si128((const __m128i *)(p + i)));
        x1 = _mm_xor_si128(fold(x1, k512), _mm_loadu_si128((const __m128i *)(p + i + 16)));
        x2 = _mm_xor_si128(fold(x2, k512), _mm_loadu_si128((const __m128i *)(p + i + 32)));
        x3 = _mm_xor_si128(fold(x3, k512), _mm_loadu_si128((const __m128i *)(p + i + 48)));
    }
    __m128i x = _mm_xor_si128(fold(x0, k128), x1);
    x = _mm_xor_si128(fold(x, k128), x2);
    x = _mm_xor_si128(fold(x, k128), x3);
    for (; i + 16 <= n; i += 16) x = _mm_xor_si128(fold(x, k128), _mm_loadu_si128((const __m128i *)(p + i)));
    alignas(16) uint8_t last[16];
    _mm_store_si128((__m128i *)last, x);
    *used = i;
    return step16(tables16(), last, 0);   // the folded block is a 16-byte message from register 0
}

__attribute__((target("pclmul,sse4.1"))) uint32_t fold_crc(const uint8_t *p, size_t n, uint32_t c, size_t *used) {
    __m128i x0 = _mm_loadu_si128((const __m128i *)p);
    x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int)c));   // the start register enters the first word
    return fold_crc_from(p, n, 64, x0, _mm_loadu_si128((const __m128i *)(p + 16)),
                         _mm_loadu_si128((const __m128i *)(p + 32)), _mm_loadu_si128((const __m128i *)(p + 48)), used);
}

// ---- the same, four lanes wide ----
#define FCS_AVX512 __attribute__((target("avx512f,vpclmulqdq,pclmul,sse4.1")))
FCS_AVX512 inline __m512i fold4(__m512i x, __m512i k) {
    return _mm512_xor_si512(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11));
}

FCS_AVX512 inline __m512i xor3(__m512i a, __m512i b, __m512i c) { return _mm512_ternarylogic_epi64(a, b, c, 0x96); }

// n >= 256: 256 bytes per step, then 64; the four lanes of the last 64 bytes go to fold_crc_from as
// its x0..x3 (bytes [i - 64, i)), which folds them (D = 128 apart) and finishes.
FCS_AVX512 uint32_t fold_crc_wide(const uint8_t *p, size_t n, uint32_t c, size_t *used) {
    const FoldK &K = fold_k();
    const __m512i k2048 = _mm512_broadcast_i32x4(_mm_load_si128((const __m128i *)K.k2048));
    const __m512i k512 = _mm512_broadcast_i32x4(_mm_load_si128((const __m128i *)K.k512));
    __m512i x0 = _mm512_loadu_si512(p), x1 = _mm512_loadu_si512(p + 64), x2 = _mm512_loadu_si512(p + 128),
            x3 = _mm512_loadu_si512(p + 192);
    x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)c)));   // start register
    size_t i = 256;
    for (; i + 256 <= n; i += 256) {
        x0 = _mm512_xor_si512(fold4(x0, k2048), _mm512_loadu_si512(p + i));
        x1 = _mm512_xor_si512(fold4(x1, k2048), _mm512_loadu_si512(p + i + 64));
        x2 = _mm512_xor_si512(fold4(x2, k2048), _mm512_loadu_si512(p + i + 128));
        x3 = _mm512_xor_si512(fold4(x3, k2048), _mm512_loadu_si512(p + i + 192));
    }
    __m512i x = xor3(fold4(x0, k512), x1, _mm512_setzero_si512());
    x = _mm512_xor_si512(fold4(x, k512), x2);
    x = _mm512_xor_si512(fold4(x, k512), x3);
    for (; i + 64 <= n; i += 64) x = _mm512_xor_si512(fold4(x, k512), _mm512_loadu_si512(p + i));
    return fold_crc_from(p, n, i, _mm512_extracti32x4_epi32(x, 0), _mm512_extracti32x4_epi32(x, 1),
                         _mm512_extracti32x4_epi32(x, 2), _mm512_extracti32x4_epi32(x, 3), used);
}
#undef FCS_AVX512

// The widest form the CPU has; NSTACK_FCS_HOST_CRC=tables or =pclmul selects a narrower one (tests
// run every form through the C ABI).
enum Form { kTables, kPclmul, kWide };
Form host_form() {
    static const Form f = [] {
        const char *e = std::getenv("NSTACK_FCS_HOST_CRC");
        if ((e && !std::strcmp(e, "tables")) || !__builtin_cpu_supports("pclmul") || !__builtin_cpu_supports("sse4.1"))
            return kTables;
        if ((e && !std::strcmp(e, "pclmul")) || !__builtin_cpu_supports("avx512f") ||
            !__builtin_cpu_supports("vpclmulqdq"))
            return kPclmul;
        return kWide;
    }();
    return f;
}

}  // namespace

uint32_t host_crc32(const void *data, size_t bsize) {
    const uint8_t *p = static_cast<const uint8_t *>(data);
    uint32_t c = 0xFFFFFFFFu;
    if (bsize >= 64) {
        const Form f = host_form();
        if (f != kTables) {
            size_t used = 0;
            c = f == kWide && bsize >= 256 ? fold_crc_wide(p, bsize, c, &used) : fold_crc(p, bsize, c, &used);
            p += used;
            bsize -= used;
        }
    }
    return ~tables_crc(p, bsize, c);
}

uint32_t host_crc32_tables(const void *data, size_t bsize) {
    return ~tables_crc(static_cast<const uint8_t *>(data), bsize, 0xFFFFFFFFu);
}

}  // namespace fcs

extern "C" uint32_t fcs_host_crc32(const void *data, size_t bsize) {
    if (!data && bsize) return 0;   // no error channel: a null buffer has no CRC
    return fcs::host_crc32(data, bsize);
}
