// fcs_pcap.cpp — classic libpcap files <-> the engine's batch layout (include/nstack_pcap.h;
// fixtures and captured traffic driving the GPU engine reproducibly).
// Host code only: parsing and packing; no CRC is computed here.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>

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

// A pcap file mapped read-only, global header validated. Records are parsed straight from the
// mapping: no per-record read or seek calls.
struct Mapped {
    const uint8_t *p = nullptr;
    uint64_t size = 0;
    bool swapped = false;
    uint32_t linktype = 0;
    ~Mapped() {
        if (p && size) munmap((void *)p, size);
    }
    uint32_t u32(uint64_t at) const {
        uint32_t v;
        std::memcpy(&v, p + at, 4);
        return swapped ? bswap32(v) : v;
    }
};

int map_pcap(const char *path, Mapped *m) {
    if (!path) return fcs::set_error(EINVAL, "null path");
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return fcs::set_error(errno ? errno : EIO, "%s: %s", path, std::strerror(errno));
    struct stat st;
    if (fstat(fd, &st) != 0) {
        const int e = errno;
        close(fd);
        return fcs::set_error(e ? e : EIO, "%s: %s", path, std::strerror(e));
    }
    m->size = (uint64_t)st.st_size;
    if (m->size < 24) {
        close(fd);
        m->size = 0;
        return fcs::set_error(EINVAL, "%s: short pcap header", path);
    }
    void *p = mmap(nullptr, m->size, PROT_READ, MAP_PRIVATE, fd, 0);
    const int e = errno;
    close(fd);
    if (p == MAP_FAILED) {
        m->size = 0;
        return fcs::set_error(e ? e : EIO, "%s: mmap: %s", path, std::strerror(e));
    }
    m->p = (const uint8_t *)p;
    madvise(p, m->size, MADV_SEQUENTIAL);
    uint32_t magic;
    std::memcpy(&magic, m->p, 4);
    if (magic == kMagicPcapng) return fcs::set_error(EPROTONOSUPPORT, "%s: pcapng is not supported", path);
    if (magic != kMagicUs && magic != kMagicNs && magic != kMagicUsSwapped && magic != kMagicNsSwapped)
        return fcs::set_error(EINVAL, "%s: not a pcap file (magic 0x%08X)", path, magic);
    m->swapped = (magic == kMagicUsSwapped || magic == kMagicNsSwapped);
    m->linktype = m->u32(20);
    return 0;
}

// Record header at *pos: 1 = got one (*pos moves past header and data), 0 = clean end of file,
// <0 = -errno.
int next_record(const Mapped &m, const char *path, uint64_t n, uint64_t *pos, uint64_t *data, uint32_t *incl,
                uint32_t *orig) {
    if (*pos == m.size) return 0;
    if (m.size - *pos < 16) return fcs::set_error(EINVAL, "%s: truncated record header", path);
    *incl = m.u32(*pos + 8);
    *orig = m.u32(*pos + 12);
    if (*incl > kMaxRecord) return fcs::set_error(EINVAL, "%s: record of %u bytes", path, *incl);
    *data = *pos + 16;
    if (*incl > m.size - *data)
        return fcs::set_error(EINVAL, "%s: truncated record %llu", path, (unsigned long long)n);
    *pos = *data + *incl;
    return 1;
}

}  // namespace

extern "C" {

int fcs_pcap_scan(const char *path, uint64_t *frames, uint64_t *bytes, uint32_t *linktype,
                  uint64_t *truncated) {
    Mapped m;
    int rc = map_pcap(path, &m);
    if (rc) return rc;
    uint64_t n = 0, b = 0, tr = 0, pos = 24;
    for (;;) {
        uint64_t data = 0;
        uint32_t incl = 0, orig = 0;
        rc = next_record(m, path, n, &pos, &data, &incl, &orig);
        if (rc < 0) return rc;
        if (rc == 0) break;
        n++;
        b += incl;
        tr += incl < orig;
    }
    if (frames) *frames = n;
    if (bytes) *bytes = b;
    if (linktype) *linktype = m.linktype;
    if (truncated) *truncated = tr;
    return 0;
}

int64_t fcs_pcap_read(const char *path, uint8_t *arena, uint64_t arena_bytes, uint64_t *off,
                      uint32_t *len, uint64_t max_frames) {
    if (max_frames && (!arena || !off || !len)) return fcs::set_error(EINVAL, "null pointer");
    Mapped m;
    int rc = map_pcap(path, &m);
    if (rc) return rc;
    // pass 1: where every record's bytes are and where they go (packed in file order)
    std::vector<uint64_t> src;
    uint64_t n = 0, pos = 24, dst = 0;
    while (n < max_frames) {
        uint64_t data = 0;
        uint32_t incl = 0, orig = 0;
        rc = next_record(m, path, n, &pos, &data, &incl, &orig);
        if (rc < 0) return rc;
        if (rc == 0) break;
        if (incl > arena_bytes - dst)
            return fcs::set_error(ENOSPC, "%s: record %llu (%u B) does not fit the %llu-byte arena", path,
                                  (unsigned long long)n, incl, (unsigned long long)arena_bytes);
        src.push_back(data);
        off[n] = dst;
        len[n] = incl;
        dst += incl;
        n++;
    }
    // pass 2: copy, split by bytes over a few threads for large captures (one core copies far
    // below the rate the GPU takes the batch at)
    const uint64_t kPerThread = 64ull << 20;
    const unsigned nth = (unsigned)std::min<uint64_t>(8, std::max<uint64_t>(1, dst / kPerThread));
    auto copy = [&](uint64_t i0, uint64_t i1) {
        for (uint64_t i = i0; i < i1; i++)
            if (len[i]) std::memcpy(arena + off[i], m.p + src[i], len[i]);
    };
    if (nth == 1) {
        copy(0, n);
    } else {
        std::vector<std::thread> th;
        uint64_t i = 0;
        for (unsigned t = 0; t < nth; t++) {
            const uint64_t goal = dst * (t + 1) / nth;   // records until this many bytes are covered
            uint64_t e = i;
            while (e < n && (t + 1 == nth || off[e] < goal)) e++;
            th.emplace_back(copy, i, e);
            i = e;
        }
        for (auto &x : th) x.join();
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
