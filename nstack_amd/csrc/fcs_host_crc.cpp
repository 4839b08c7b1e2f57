// fcs_host_crc.cpp — host CRC-32 for the failure paths of the drop-in and the TX/RX queues only
// (fcs_host_crc.hpp).
//
// Slice-by-16: sixteen 256-entry tables, table k advancing a byte past k further zero bytes, so
// one step folds 16 input bytes with 16 independent lookups. The tables are derived from the
// reflected polynomial 0xEDB88320 (the operator the reference's nibble table folds,
// src/ether_fcs.c:7-10); the register starts at ~0 and is complemented at the end, which is what
// the reference's complement-folded table computes ("123456789" -> 0xCBF43926).
// A single host thread: this path exists for correctness when no GPU answers, not for speed.
#include "fcs_host_crc.hpp"

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

}  // namespace

uint32_t host_crc32(const void *data, size_t bsize) {
    const Slice16 &s = tables16();
    const uint8_t *p = static_cast<const uint8_t *>(data);
    uint32_t c = 0xFFFFFFFFu;
    while (bsize >= 16) {
        const uint32_t a = le32(p) ^ c, b = le32(p + 4), d = le32(p + 8), e = le32(p + 12);
        c = s.t[15][a & 0xFF] ^ s.t[14][(a >> 8) & 0xFF] ^ s.t[13][(a >> 16) & 0xFF] ^ s.t[12][a >> 24] ^
            s.t[11][b & 0xFF] ^ s.t[10][(b >> 8) & 0xFF] ^ s.t[9][(b >> 16) & 0xFF] ^ s.t[8][b >> 24] ^
            s.t[7][d & 0xFF] ^ s.t[6][(d >> 8) & 0xFF] ^ s.t[5][(d >> 16) & 0xFF] ^ s.t[4][d >> 24] ^
            s.t[3][e & 0xFF] ^ s.t[2][(e >> 8) & 0xFF] ^ s.t[1][(e >> 16) & 0xFF] ^ s.t[0][e >> 24];
        p += 16;
        bsize -= 16;
    }
    while (bsize--) c = (c >> 8) ^ s.t[0][(c ^ *p++) & 0xFFu];
    return ~c;
}

}  // namespace fcs
