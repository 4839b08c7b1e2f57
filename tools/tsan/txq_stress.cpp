// txq_stress.cpp — ThreadSanitizer stress of the TX queue (include/nstack_txq.h): 6 producers with
// ether_send semantics and 3 fire-and-forget producers on one queue, then flush/stats/destroy.
// Every frame must be sunk exactly once and every sync caller must get its frame_size back.
//   usage: txq_stress <max_batch> <flush_usec>      (build and run: tools/tsan/run.sh)
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include "nstack_txq.h"
static std::atomic<uint64_t> sunk{0};
static void sink(void *, uint8_t *const *f, const uint32_t *sz, int *res, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) res[i] = (int)sz[i];
    sunk += n;
}
int main(int argc, char **argv) {
    const uint32_t CAP = atoi(argv[1]), LIN = atoi(argv[2]);
    const uint8_t mac[6] = {2,0,0,0,0,1}, dst[6] = {2,0,0,0,0,2};
    { const uint32_t cap = CAP, linger = LIN;
        sunk = 0;
        fcs_txq_t *q = fcs_txq_create(mac, cap, linger, sink, nullptr);
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        const int per = 400;
        for (int k = 0; k < 6; k++) th.emplace_back([&, k] {
            uint8_t buf[1500]; for (int i = 0; i < per; i++) { int L = (i * 31 + k) % 1400;
                int r = fcs_txq_send(q, dst, 0x0800, buf, L); if (r != 14 + (L < 56 ? 56 : L) + 4) bad++; } });
        for (int k = 0; k < 3; k++) th.emplace_back([&] {
            uint8_t buf[1500]; for (int i = 0; i < per; i++) if (fcs_txq_send_async(q, dst, 0x0806, buf, i % 200) <= 0) bad++; });
        for (auto &t : th) t.join();
        fcs_txq_flush(q);
        uint64_t fr, ba, er; fcs_txq_stats(q, &fr, &ba, &er);
        fcs_txq_destroy(q);
        std::printf("cap %u linger %u: frames %llu batches %llu errors %llu sunk %llu bad %d\n", cap, linger,
                    (unsigned long long)fr, (unsigned long long)ba, (unsigned long long)er, (unsigned long long)sunk.load(), bad.load());
        if (fr != 9u * per || er || sunk != 9u * per || bad) return 1;
    }
    return 0;
}
