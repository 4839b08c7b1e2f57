// rxq_stress.cpp — sanitizer stress of the RX queue (include/nstack_rxq.h) over an AF_UNIX datagram
// socketpair: a writer thread sends frames with their FCS trailer (some corrupted, some runts or
// oversize, some echoes of the receiver's own MAC) while the reader takes them one ether_receive
// call at a time with varying buffer sizes. Every good frame must come out once, in order, with
// the reference's header and payload semantics (src/linux/ether.c:180-212), and the queue's drop
// counters must match what was sent.
//   usage: rxq_stress <max_batch> <host_max|-1> [frames]   (build and run: tools/tsan/run.sh)
// host_max (fcs_rxq_set_host_max): -1 = the default; 0 = every batch through the (stubbed) GPU check;
// -2 = another thread switches it between 0 and 1 MiB while the reader receives.
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "nstack_fcs.h"
#include "nstack_rxq.h"

namespace fcs { uint32_t host_crc32(const void *data, size_t bsize); }

enum Kind { kGood, kBadFcs, kRunt, kOversize, kEcho };
struct Sent {
    Kind kind;
    std::vector<uint8_t> frame;   // header + payload (+ trailer)
};

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const uint32_t cap = (uint32_t)atoi(argv[1]);
    const long long hmax = atoll(argv[2]);
    const int nframes = argc > 3 ? atoi(argv[3]) : 3000;
    const uint8_t own[6] = {2, 0, 0, 0, 0, 9}, peer[6] = {2, 0, 0, 0, 0, 7};
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv)) { perror("socketpair"); return 2; }
    const int sndbuf = 4 << 20;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof sndbuf);
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &sndbuf, sizeof sndbuf);

    std::mt19937_64 rng(cap * 1000003ull + (uint64_t)(hmax + 1));
    std::vector<Sent> sent(nframes);
    for (int i = 0; i < nframes; i++) {
        Sent &s = sent[i];
        const uint32_t r = (uint32_t)(rng() % 100);
        s.kind = i == nframes - 1 ? kGood : r < 70 ? kGood : r < 80 ? kBadFcs : r < 86 ? kRunt : r < 92 ? kOversize : kEcho;
        uint32_t len;   // covered bytes (header + payload)
        if (s.kind == kRunt) len = (uint32_t)(rng() % 14);
        else if (s.kind == kOversize) len = 1515 + (uint32_t)(rng() % 500);
        else len = 15 + (uint32_t)(rng() % 1500);   // payload >= 1: ether_receive's 0 also means "nothing queued"
        s.frame.resize(len + 4);
        for (uint32_t k = 0; k < len; k++) s.frame[k] = (uint8_t)rng();
        std::memcpy(&s.frame[0], own, std::min<uint32_t>(len, 6));
        if (len >= 12) std::memcpy(&s.frame[6], s.kind == kEcho ? own : peer, 6);
        if (len >= 14) { s.frame[12] = 0x08; s.frame[13] = (uint8_t)i; }
        const uint32_t c = fcs::host_crc32(s.frame.data(), len);
        std::memcpy(&s.frame[len], &c, 4);
        if (s.kind == kBadFcs) s.frame[rng() % (len + 4)] ^= (uint8_t)(1u << (rng() % 8));
    }

    std::thread writer([&] {
        for (const Sent &s : sent)
            if (send(sv[0], s.frame.data(), s.frame.size(), 0) != (ssize_t)s.frame.size()) { perror("send"); std::abort(); }
    });

    fcs_rxq_t *q = fcs_rxq_create(sv[1], own, cap, FCS_RXQ_TRAILER);
    if (!q) { fprintf(stderr, "create failed\n"); return 2; }
    if (hmax >= 0) fcs_rxq_set_host_max(q, (uint64_t)hmax);
    std::atomic<bool> done{false};
    std::thread toggler([&] {
        for (uint64_t k = 0; hmax == -2 && !done.load(); k++) {
            fcs_rxq_set_host_max(q, (k & 1) << 20);
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    });
    uint64_t want_bad = 0, want_echo = 0, want_drop = 0;
    std::vector<const Sent *> good;
    for (const Sent &s : sent) {
        if (s.kind == kGood) good.push_back(&s);
        else if (s.kind == kBadFcs) (s.frame.size() - 4 >= 12 && !std::memcmp(&s.frame[6], own, 6)) ? want_echo++ : want_bad++;
        else if (s.kind == kEcho) want_echo++;
        else want_drop++;
    }
    int bad = 0;
    std::vector<uint8_t> buf(1600);
    for (size_t g = 0; g < good.size() && !bad; g++) {
        const size_t bsize = (size_t)(rng() % 4 == 0 ? 0 : rng() % 1600);
        fcs_ether_hdr h{};
        int r;
        while ((r = fcs_rxq_receive(q, &h, bsize ? buf.data() : nullptr, bsize)) == 0) {}
        const std::vector<uint8_t> &f = good[g]->frame;
        const int payload = (int)f.size() - 4 - 14;
        if (r != payload || std::memcmp(h.h_dst, &f[0], 6) || std::memcmp(h.h_src, &f[6], 6) ||
            h.h_proto != (uint16_t)((f[12] << 8) | f[13]) ||
            (bsize && std::memcmp(buf.data(), &f[14], std::min<size_t>((size_t)payload, bsize)))) {
            fprintf(stderr, "frame %zu: got %d want %d\n", g, r, payload);
            bad = 1;
        }
    }
    writer.join();
    done = true;
    toggler.join();
    uint64_t frames, nbad, echo, drop, batches, small, gpu, hb, hf;
    fcs_rxq_stats(q, &frames, &nbad, &echo, &drop, &batches);
    fcs_rxq_small_batches(q, &small, nullptr, &gpu);
    fcs_rxq_fallbacks(q, &hb, &hf);
    printf("cap %u host_max %lld: frames %llu batches %llu (host %llu gpu %llu fallback %llu) bad %llu echo %llu drop %llu\n",
           cap, hmax, (unsigned long long)frames, (unsigned long long)batches, (unsigned long long)small,
           (unsigned long long)gpu, (unsigned long long)hb, (unsigned long long)nbad, (unsigned long long)echo,
           (unsigned long long)drop);
    if (frames != (uint64_t)nframes || nbad != want_bad || echo != want_echo || drop != want_drop) {
        fprintf(stderr, "counters: want bad %llu echo %llu drop %llu\n", (unsigned long long)want_bad,
                (unsigned long long)want_echo, (unsigned long long)want_drop);
        bad = 1;
    }
    fcs_rxq_destroy(q);
    close(sv[0]);
    close(sv[1]);
    return bad;
}
