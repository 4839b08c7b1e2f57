// pcap_fuzz.cpp — mutation fuzz of the pcap reader (nstack_amd/csrc/fcs_pcap.cpp) under the
// sanitizers: a valid capture written by fcs_pcap_write is corrupted (bit flips, overwritten record
// lengths, truncation, both byte orders, a pcapng magic) and fed to fcs_pcap_scan / fcs_pcap_read.
// Every call must return a count or -errno without reading or writing out of bounds, and an intact
// file must read back byte for byte.
//   usage: pcap_fuzz [iterations]   (build and run: tools/tsan/run.sh)
#include <unistd.h>

#include <cerrno>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "nstack_pcap.h"

namespace fcs {   // the engine's error setter (fcs_engine.cpp), reduced to its return value
int set_error(int err, const char *, ...) { return -err; }
}  // namespace fcs

static std::vector<uint8_t> slurp(const std::string &p) {
    std::vector<uint8_t> v;
    if (FILE *f = std::fopen(p.c_str(), "rb")) {
        uint8_t b[4096];
        size_t k;
        while ((k = std::fread(b, 1, sizeof b, f)) > 0) v.insert(v.end(), b, b + k);
        std::fclose(f);
    }
    return v;
}

static void spit(const std::string &p, const std::vector<uint8_t> &v) {
    FILE *f = std::fopen(p.c_str(), "wb");
    if (!f) std::abort();
    if (!v.empty() && std::fwrite(v.data(), 1, v.size(), f) != v.size()) std::abort();
    std::fclose(f);
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
    const char *tmp = std::getenv("TMPDIR") ? std::getenv("TMPDIR") : "/tmp";
    const std::string path = std::string(tmp) + "/pcap_fuzz_" + std::to_string(getpid()) + ".pcap";
    std::mt19937_64 rng(12345);
    // a valid capture: 40 frames of 0..1600 bytes
    const uint64_t nf = 40;
    std::vector<uint64_t> off(nf);
    std::vector<uint32_t> len(nf);
    std::vector<uint8_t> arena;
    for (uint64_t i = 0; i < nf; i++) {
        off[i] = arena.size();
        len[i] = (uint32_t)(rng() % 1601);
        for (uint32_t k = 0; k < len[i]; k++) arena.push_back((uint8_t)rng());
    }
    if (fcs_pcap_write(path.c_str(), arena.data(), off.data(), len.data(), nf, 1)) return 2;
    const std::vector<uint8_t> good = slurp(path);
    {   // intact: scan and read back
        uint64_t frames = 0, bytes = 0, tr = 0;
        uint32_t lt = 0;
        std::vector<uint8_t> a2(arena.size());
        std::vector<uint64_t> o2(nf);
        std::vector<uint32_t> l2(nf);
        if (fcs_pcap_scan(path.c_str(), &frames, &bytes, &lt, &tr) || frames != nf || bytes != arena.size() || lt != 1 ||
            fcs_pcap_read(path.c_str(), a2.data(), a2.size(), o2.data(), l2.data(), nf) != (int64_t)nf || a2 != arena ||
            l2 != len || o2 != off) {
            std::fprintf(stderr, "intact capture did not read back\n");
            return 1;
        }
    }
    uint64_t ok = 0, err = 0;
    for (int it = 0; it < iters; it++) {
        std::vector<uint8_t> v = good;
        switch (it % 6) {
        case 0:   // bit flips anywhere
            for (int k = 0; k < 1 + (int)(rng() % 8); k++) v[rng() % v.size()] ^= (uint8_t)(1u << (rng() % 8));
            break;
        case 1: {   // a record length field overwritten (incl or orig of some record, or a random spot)
            const size_t at = 24 + (rng() % (v.size() - 28));
            const uint32_t x = (uint32_t)rng() >> (rng() % 32);
            std::memcpy(&v[at], &x, 4);
            break;
        }
        case 2:   // truncated anywhere (header included)
            v.resize(rng() % v.size());
            break;
        case 3:   // the other byte order's magic with unchanged fields
            v[0] = 0xD4, v[1] = 0xC3, v[2] = 0xB2, v[3] = 0xA1;
            break;
        case 4:   // pcapng
            v[0] = 0x0A, v[1] = 0x0D, v[2] = 0x0D, v[3] = 0x0A;
            break;
        default:   // garbage appended
            for (int k = 0; k < (int)(rng() % 40); k++) v.push_back((uint8_t)rng());
        }
        spit(path, v);
        uint64_t frames = 0, bytes = 0;
        const int rc = fcs_pcap_scan(path.c_str(), &frames, &bytes, nullptr, nullptr);
        // read into buffers sized from the scan when it succeeded, else small random ones
        const uint64_t cap_frames = rc == 0 ? frames : rng() % 64;
        const uint64_t cap_bytes = rc == 0 ? (rng() % 2 ? bytes : bytes / 2) : rng() % 70000;
        std::vector<uint8_t> a2(cap_bytes + 1);
        std::vector<uint64_t> o2(cap_frames + 1);
        std::vector<uint32_t> l2(cap_frames + 1);
        const int64_t r = fcs_pcap_read(path.c_str(), a2.data(), cap_bytes, o2.data(), l2.data(), cap_frames);
        if (r >= 0) {
            ok++;
            for (int64_t i = 0; i < r; i++)
                if (o2[i] + l2[i] > cap_bytes) {
                    std::fprintf(stderr, "record %lld outside the arena\n", (long long)i);
                    return 1;
                }
        } else {
            err++;
        }
    }
    unlink(path.c_str());
    std::printf("pcap fuzz: %d inputs, %llu read, %llu rejected\n", iters, (unsigned long long)ok,
                (unsigned long long)err);
    return 0;
}
