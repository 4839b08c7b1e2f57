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
    {
        const int reps = 2000;
        (void)ether_fcs(pag, 1514);
        const double t0 = now();
        uint32_t x = 0;
        for (int r = 0; r < reps; r++) x ^= ether_fcs(pag, 1514);
        printf("{\"path\": \"dropin_ether_fcs\", \"n\": 1, \"us_per_call\": %.1f, \"x\": %u}\n",
               (now() - t0) / reps * 1e6, x);
    }
    free(pag);
    free(len);
    fcs_host_free(pin);
    return 0;
}
