// txq_stress.cpp — ThreadSanitizer stress of the TX queue (include/nstack_txq.h): 6 producers with
// ether_send semantics and 3 fire-and-forget producers on one queue, then flush/stats/destroy.
// Every frame must be sunk exactly once, every sync caller must get its frame_size back, and each
// fire-and-forget producer's frames must reach the sink in the order it queued them.
//   usage: txq_stress <max_batch> <flush_usec> [host_max]   (build and run: tools/tsan/run.sh)
// host_max (fcs_txq_set_host_max): absent = the default (sync callers compute their own FCS, small
// fire-and-forget batches on the flusher); 0 = every frame through the (stubbed) GPU step.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include "nstack_txq.h"
static std::atomic<uint64_t> sunk{0};
static uint32_t last_seen[8];      // per async producer: last counter the sink saw (sink: one thread)
static std::atomic<int> reordered{0};
static void sink(void *, uint8_t *const *f, const uint32_t *sz, int *res, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        res[i] = (int)sz[i];
        if (f[i][12] == 0x08 && f[i][13] == 0x06) {   // async producer: payload = (thread, counter)
            uint32_t t = f[i][14], c;
            std::memcpy(&c, f[i] + 15, 4);
            if (c <= last_seen[t]) reordered++;
            last_seen[t] = c;
        }
    }
    sunk += n;
}
int main(int argc, char **argv) {
    const uint32_t CAP = atoi(argv[1]), LIN = atoi(argv[2]);
    const long long HMAX = argc > 3 ? atoll(argv[3]) : -1;
    const uint8_t mac[6] = {2,0,0,0,0,1}, dst[6] = {2,0,0,0,0,2};
    { const uint32_t cap = CAP, linger = LIN;
        sunk = 0;
        fcs_txq_t *q = fcs_txq_create(mac, cap, linger, sink, nullptr);
        if (HMAX >= 0) fcs_txq_set_host_max(q, (uint64_t)HMAX);
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        const int per = 400;
        for (int k = 0; k < 6; k++) th.emplace_back([&, k] {
            uint8_t buf[1500]; for (int i = 0; i < per; i++) { int L = (i * 31 + k) % 1400;
                int r = fcs_txq_send(q, dst, 0x0800, buf, L); if (r != 14 + (L < 56 ? 56 : L) + 4) bad++; } });
        for (int k = 0; k < 3; k++) th.emplace_back([&, k] {
            uint8_t buf[1500];
            for (int i = 0; i < per; i++) {
                const uint32_t c = i + 1;
                buf[0] = (uint8_t)k;
                std::memcpy(buf + 1, &c, 4);
                if (fcs_txq_send_async(q, dst, 0x0806, buf, 5 + i % 200) <= 0) bad++;
            } });
        for (auto &t : th) t.join();
        fcs_txq_flush(q);
        uint64_t fr, ba, er; fcs_txq_stats(q, &fr, &ba, &er);
        fcs_txq_destroy(q);
        std::printf("cap %u linger %u: frames %llu batches %llu errors %llu sunk %llu bad %d\n", cap, linger,
                    (unsigned long long)fr, (unsigned long long)ba, (unsigned long long)er, (unsigned long long)sunk.load(), bad.load());
        if (reordered) std::printf("  %d frames left out of their producer's order\n", reordered.load());
        if (fr != 9u * per || er || sunk != 9u * per || bad || reordered) return 1;
        std::memset(last_seen, 0, sizeof last_seen);
    }
    return 0;
}
