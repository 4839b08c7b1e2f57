/* tx_crossover.c — the TX queue's GPU minimum (fcs_txq_set_host_max), measured: for batches of n
 * frames in the queue's own layout (fcs_host_alloc arena, 1536-B slots), the median time of one GPU
 * step (ether_fcs_tx_batch_host, what the flusher calls) against the library's host CRC over the same
 * frames on one thread (fcs_host_crc32 + the little-endian store, what the flusher does below the
 * minimum). Prints one JSON line per (covered length, n) and, per length, the smallest n at which the
 * GPU step is faster. Both paths must write the same FCSs (checked).
 *   tools/tx_crossover [reps]
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nstack_fcs.h"

static double now_us(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static int cmp(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return x < y ? -1 : x > y;
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 300;
    const int ns[] = {1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512, 1024};
    const int nn = sizeof ns / sizeof ns[0], NMAX = 1024, STRIDE = 1536;
    const uint32_t lens[] = {60, 576, 1514};
    if (fcs_engine_init(1) < 0) return fprintf(stderr, "engine: %s\n", fcs_last_error()), 1;
    uint8_t *arena = fcs_host_alloc((uint64_t)NMAX * STRIDE), *copy = malloc((size_t)NMAX * STRIDE);
    uint64_t *off = malloc(NMAX * 8);
    uint32_t *len = malloc(NMAX * 4);
    double *t = malloc(R * sizeof(double));
    if (!arena || !copy) return fprintf(stderr, "alloc failed\n"), 1;
    for (int i = 0; i < NMAX * STRIDE; i++) arena[i] = (uint8_t)(i * 131 + (i >> 9));
    for (int i = 0; i < NMAX; i++) off[i] = (uint64_t)i * STRIDE;
    for (int li = 0; li < 3; li++) {
        const uint32_t L = lens[li];
        int cross = -1;
        for (int i = 0; i < NMAX; i++) len[i] = L;
        for (int k = 0; k < nn; k++) {
            const int n = ns[k];
            const uint64_t span = (uint64_t)(n - 1) * STRIDE + L + 4;
            for (int w = 0; w < 20; w++) ether_fcs_tx_batch_host(arena, span, off, len, n);
            for (int r = 0; r < R; r++) {
                const double a = now_us();
                if (ether_fcs_tx_batch_host(arena, span, off, len, n)) return fprintf(stderr, "gpu: %s\n", fcs_last_error()), 1;
                t[r] = now_us() - a;
            }
            qsort(t, R, sizeof *t, cmp);
            const double gpu = t[R / 2], gpu90 = t[R * 9 / 10];
            memcpy(copy, arena, span);
            for (int r = 0; r < R; r++) {
                const double a = now_us();
                for (int i = 0; i < n; i++) {
                    const uint32_t c = fcs_host_crc32(copy + off[i], L);
                    memcpy(copy + off[i] + L, &c, 4);
                }
                t[r] = now_us() - a;
            }
            qsort(t, R, sizeof *t, cmp);
            const double host = t[R / 2];
            int same = 1;
            for (int i = 0; i < n; i++) same &= !memcmp(copy + off[i] + L, arena + off[i] + L, 4);
            if (!same) return fprintf(stderr, "GPU and host FCS differ at n=%d L=%u\n", n, L), 1;
            if (cross < 0 && gpu < host) cross = n;
            printf("{\"covered\": %u, \"n\": %d, \"bytes\": %llu, \"gpu_us_p50\": %.2f, \"gpu_us_p90\": %.2f, "
                   "\"host_us_p50\": %.2f, \"host_ns_per_byte\": %.3f}\n", L, n, (unsigned long long)n * L, gpu,
                   gpu90, host, host * 1e3 / ((double)n * L));
            fflush(stdout);
        }
        printf("{\"covered\": %u, \"crossover_frames\": %d, \"crossover_bytes\": %llu}\n", L, cross,
               cross > 0 ? (unsigned long long)cross * L : 0ull);
    }
    fcs_host_free(arena);
    return 0;
}
