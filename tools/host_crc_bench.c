/* host_crc_bench.c — per-call cost of the library's host CRC (fcs_host_crc32, fcs_host_crc.cpp) at the
 * lengths the TX/RX queues hand it (60 .. 1518 B), 9000 B and 64 KiB: cache-hot, one thread, in the
 * form NSTACK_FCS_HOST_CRC selects (tables | pclmul | unset: the widest the CPU has). One JSON line
 * per length. Measurement tool only (tools/Makefile builds it against the product library). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "nstack_fcs.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(void) {
    static const size_t lens[] = {60, 64, 128, 256, 576, 1514, 1518, 9000, 65536};
    const size_t cap = 1 << 17;
    uint8_t *buf = malloc(cap);
    if (!buf) return 1;
    for (size_t i = 0; i < cap; i++) buf[i] = (uint8_t)((i * 2654435761u) >> 13);
    const char *form = getenv("NSTACK_FCS_HOST_CRC");
    for (size_t k = 0; k < sizeof lens / sizeof lens[0]; k++) {
        const size_t L = lens[k];
        size_t reps = (size_t)(600e6 / (double)L);
        if (reps < 20000) reps = 20000;
        uint32_t acc = 0;
        for (size_t r = 0; r < 2000; r++) acc ^= fcs_host_crc32(buf + (r & 63), L);
        double best = 1e30;
        for (int trial = 0; trial < 3; trial++) {   /* best of three: the box's other tenants */
            const double t0 = now_s();
            for (size_t r = 0; r < reps; r++) acc ^= fcs_host_crc32(buf + (r & 63), L);
            const double s = now_s() - t0;
            if (s < best) best = s;
        }
        printf("{\"form\": \"%s\", \"len\": %zu, \"ns_per_call\": %.2f, \"GB_s\": %.2f, \"sink\": %u}\n",
               form ? form : "widest", L, best / (double)reps * 1e9, (double)L * (double)reps / best / 1e9, acc & 1);
    }
    free(buf);
    return 0;
}
