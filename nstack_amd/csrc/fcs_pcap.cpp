// fcs_pcap.cpp — classic libpcap files <-> the engine's batch layout (include/nstack_pcap.h;
// fixtures and captured traffic driving the GPU engine reproducibly).
// Host code only: parsing and packing; no CRC is computed here.
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <memory>

#include "../../include/nstack_pcap.h"
#include "fcs_error.hpp"

namespace {

constexpr uint32_t kMagicUs = 0xA1B2C3D4u, kMagicNs = 0xA1B23C4Du;
constexpr uint32_t kMagicUsSwapped = 0xD4C3B2A1u, kMagicNsSwapped = 0x4D3CB2A1u;
constexpr uint32_t kMagicPcapng = 0x0A0D0D0Au;
constexpr uint32_t kMaxRecord = 256u << 20;   // sanity bound on one record's captured length

struct FileCloser {
    void operator()(FILE *f) const {
        if (f) std::fclose(f);
    }
};
using File = std::unique_ptr<FILE, FileCloser>;

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Opens `path`, validates the 24-byte global header; returns 0 or -errno.
int open_pcap(const char *path, File *out, bool *swapped, uint32_t *linktype, uint32_t *snaplen) {
    if (!path) return fcs::set_error(EINVAL, "null path");
    File f(std::fopen(path, "rb"));
    if (!f) return fcs::set_error(errno ? errno : EIO, "%s: %s", path, std::strerror(errno));
    uint32_t h[6];
    if (std::fread(h, 4, 6, f.get()) != 6) return fcs::set_error(EINVAL, "%s: short pcap header", path);
    const uint32_t m = h[0];
    if (m == kMagicPcapng) return fcs::set_error(EPROTONOSUPPORT, "%s: pcapng is not supported", path);
    if (m != kMagicUs && m != kMagicNs && m != kMagicUsSwapped && m != kMagicNsSwapped)
        return fcs::set_error(EINVAL, "%s: not a pcap file (magic 0x%08X)", path, m);
    *swapped = (m == kMagicUsSwapped || m == kMagicNsSwapped);
    *snaplen = *swapped ? bswap32(h[4]) : h[4];
    *linktype = *swapped ? bswap32(h[5]) : h[5];
    *out = std::move(f);
    return 0;
}

// Reads the next 16-byte record header: 1 = got one, 0 = clean end of file, <0 = -errno.
int next_record(FILE *f, bool swapped, const char *path, uint32_t *incl, uint32_t *orig) {
    uint32_t r[4];
    const size_t got = std::fread(r, 4, 4, f);
    if (got == 0 && std::feof(f)) return 0;
    if (got != 4) return fcs::set_error(EINVAL, "%s: truncated record header", path);
    *incl = swapped ? bswap32(r[2]) : r[2];
    *orig = swapped ? bswap32(r[3]) : r[3];
    if (*incl > kMaxRecord) return fcs::set_error(EINVAL, "%s: record of %u bytes", path, *incl);
    return 1;
}

}  // namespace

extern "C" {

int fcs_pcap_scan(const char *path, uint64_t *frames, uint64_t *bytes, uint32_t *linktype,
                  uint64_t *truncated) {
    File f;
    bool sw = false;
    uint32_t lt = 0, snap = 0;
    int rc = open_pcap(path, &f, &sw, &lt, &snap);
    if (rc) return rc;
    uint64_t n = 0, b = 0, tr = 0;
    for (;;) {
        uint32_t incl = 0, orig = 0;
        rc = next_record(f.get(), sw, path, &incl, &orig);
        if (rc < 0) return rc;
        if (rc == 0) break;
        if (std::fseek(f.get(), incl, SEEK_CUR) != 0) return fcs::set_error(EIO, "%s: seek failed", path);
        n++;
        b += incl;
        tr += incl < orig;
    }
    if (frames) *frames = n;
    if (bytes) *bytes = b;
    if (linktype) *linktype = lt;
    if (truncated) *truncated = tr;
    return 0;
}

int64_t fcs_pcap_read(const char *path, uint8_t *arena, uint64_t arena_bytes, uint64_t *off,
                      uint32_t *len, uint64_t max_frames) {
    if (max_frames && (!arena || !off || !len)) return fcs::set_error(EINVAL, "null pointer");
    File f;
    bool sw = false;
    uint32_t lt = 0, snap = 0;
    int rc = open_pcap(path, &f, &sw, &lt, &snap);
    if (rc) return rc;
    uint64_t n = 0, pos = 0;
    while (n < max_frames) {
        uint32_t incl = 0, orig = 0;
        rc = next_record(f.get(), sw, path, &incl, &orig);
        if (rc < 0) return rc;
        if (rc == 0) break;
        if (incl > arena_bytes - pos)
            return fcs::set_error(ENOSPC, "%s: record %llu (%u B) does not fit the %llu-byte arena", path,
                                  (unsigned long long)n, incl, (unsigned long long)arena_bytes);
        if (incl && std::fread(arena + pos, 1, incl, f.get()) != incl)
            return fcs::set_error(EINVAL, "%s: truncated record %llu", path, (unsigned long long)n);
        off[n] = pos;
        len[n] = incl;
        pos += incl;
        n++;
    }
    return (int64_t)n;
}

int fcs_pcap_write(const char *path, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                   uint64_t n, uint32_t linktype) {
    if (!path || (n && (!arena || !off || !len))) return fcs::set_error(EINVAL, "null pointer");
    File f(std::fopen(path, "wb"));
    if (!f) return fcs::set_error(errno ? errno : EIO, "%s: %s", path, std::strerror(errno));
    const uint32_t h[6] = {kMagicUs, 0x00040002u /* version 2.4 */, 0, 0, 65535u, linktype};
    if (std::fwrite(h, 4, 6, f.get()) != 6) return fcs::set_error(EIO, "%s: write failed", path);
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t r[4] = {(uint32_t)(i / 1000000), (uint32_t)(i % 1000000), len[i], len[i]};
        if (std::fwrite(r, 4, 4, f.get()) != 4 || (len[i] && std::fwrite(arena + off[i], 1, len[i], f.get()) != len[i]))
            return fcs::set_error(EIO, "%s: write failed at record %llu", path, (unsigned long long)i);
    }
    if (std::fflush(f.get()) != 0) return fcs::set_error(EIO, "%s: flush failed", path);
    return 0;
}

}  // extern "C"
