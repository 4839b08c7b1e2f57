/* tx_latency.c — latency breakdown of the small-batch GPU paths (measurement tool).
 *   ether_fcs_tx_host on pinned frames (zero-copy path) and on pageable frames (staged pipeline),
 *   the drop-in ether_fcs, and ether_fcs_fixed_dev on device memory (launch + kernel + sync).
 * Build: gcc -O2 tools/tx_latency.c -Iinclude -Lnstack_amd -lnstack_fcs -Wl,-rpath,'$ORIGIN/../nstack_amd'
 *        -o tools/tx_latency */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nstack_fcs.h"

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static int cmp_double(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

int main(void) {
    if (fcs_engine_init(1) < 0) return fprintf(stderr, "%s\n", fcs_last_error()), 1;
    const int ns[] = {1, 16, 128, 1024, 4096, 8192, 16384, 32768};
    const int NMAX = 32768;
    const uint64_t stride = 1518;
    uint8_t *pin = fcs_host_alloc((uint64_t)NMAX * stride);
    uint8_t *pag = malloc((uint64_t)NMAX * stride);
    uint32_t *len = malloc((uint64_t)NMAX * 4);
    for (int i = 0; i < NMAX; i++) len[i] = 1514;
    memset(pin, 7, (uint64_t)NMAX * stride);
    memset(pag, 7, (uint64_t)NMAX * stride);
    for (unsigned k = 0; k < sizeof ns / sizeof ns[0]; k++) {
        const int n = ns[k];
        const int reps = 200;
        for (int w = 0; w < 2; w++) {
            uint8_t *b = w ? pag : pin;
            ether_fcs_tx_host(b, stride, len, n);   /* warm */
            const double t0 = now();
            for (int r = 0; r < reps; r++)
                if (ether_fcs_tx_host(b, stride, len, n)) return fprintf(stderr, "%s\n", fcs_last_error()), 1;
            const double t = (now() - t0) / reps;
            printf("{\"path\": \"tx_host_%s\", \"n\": %d, \"us_per_call\": %.1f, \"Mframes_s\": %.3f}\n",
                   w ? "pageable" : "pinned", n, t * 1e6, n / t / 1e6);
        }
    }
    {   /* drop-in: <= 1536 B through the single-frame kernel, longer through the staged path */
        const uint32_t lens[] = {64, 1514, 1536, 4000};
        enum { REPS = 2000 };
        static double ts[REPS];
        for (unsigned k = 0; k < sizeof lens / sizeof lens[0]; k++) {
            uint32_t x = ether_fcs(pag, lens[k]);
            double sum = 0;
            for (int r = 0; r < REPS; r++) {
                const double t0 = now();
                x ^= ether_fcs(pag, lens[k]);
                ts[r] = now() - t0;
                sum += ts[r];
            }
            qsort(ts, REPS, sizeof ts[0], cmp_double);
            printf("{\"path\": \"dropin_ether_fcs\", \"len\": %u, \"us_per_call\": %.2f, \"p50_us\": %.2f, "
                   "\"p99_us\": %.2f, \"x\": %u}\n",
                   lens[k], sum / REPS * 1e6, ts[REPS / 2] * 1e6, ts[REPS * 99 / 100] * 1e6, x);
        }
    }
    free(pag);
    free(len);
    fcs_host_free(pin);
    return 0;
}
