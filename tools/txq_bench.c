/* txq_bench.c — rate of the batched TX call site (include/nstack_txq.h) on one GPU box.
 *
 *   tools/txq_bench [producers] [frames_per_producer] [payload|-1=random] [max_batch] [flush_usec]
 *                   [sink: null|sock] [mode: txq|async|dropin]
 *
 * txq:    P producer threads call fcs_txq_send (ether_send semantics) into one queue;
 *         the sink is either a counting null sink or a socketpair drained by a reader thread.
 * async:  the same through fcs_txq_send_async (fire-and-forget; batches fill to max_batch).
 * dropin: each producer builds the frame itself and calls the drop-in ether_fcs() per frame,
 *         then the same sink for that one frame — today's ether_send with the library linked in.
 * Prints one JSON line: frames/s, on-wire Gbit/s, mean batch size.
 * Build: gcc -O2 -pthread tools/txq_bench.c -Iinclude -Lnstack_amd -lnstack_fcs \
 *            -Wl,-rpath,'$ORIGIN/../nstack_amd' -o tools/txq_bench
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "nstack_fcs.h"
#include "nstack_txq.h"

static int P = 8, M = 20000, PAYLOAD = 1500, BATCH = 512, FLUSH_US = 0, SOCK = 0, DROPIN = 0, ASYNC = 0;
static fcs_txq_t *Q;
static int sock_tx = -1, sock_rx = -1;
static atomic_ullong sunk_frames, sunk_bytes, bad_results;
static const uint8_t MAC[6] = {2, 0, 0, 0, 0, 1};

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void null_sink(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res, uint32_t n) {
    (void)ctx;
    (void)frames;
    uint64_t b = 0;
    for (uint32_t i = 0; i < n; i++) {
        res[i] = (int)sizes[i];
        b += sizes[i];
    }
    atomic_fetch_add(&sunk_frames, n);
    atomic_fetch_add(&sunk_bytes, b);
}

static void *reader(void *arg) {
    (void)arg;
    static uint8_t buf[2048];
    for (;;) {
        ssize_t r = recv(sock_rx, buf, sizeof buf, 0);
        if (r <= 0) break;
        atomic_fetch_add(&sunk_frames, 1);
        atomic_fetch_add(&sunk_bytes, (unsigned long long)r);
    }
    return NULL;
}

static void *producer(void *arg) {
    const int t = (int)(intptr_t)arg;
    uint64_t s = 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1);
    uint8_t payload[1500], dst[6] = {2, 0, 0, 0, 1, (uint8_t)t}, frame[1518];
    for (int i = 0; i < 1500; i++) payload[i] = (uint8_t)(i * 31 + t);
    for (int i = 0; i < M; i++) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        const size_t bsize = PAYLOAD >= 0 ? (size_t)PAYLOAD : (size_t)(s % 1501);
        const size_t fs = 14 + (bsize > 56 ? bsize : 56) + 4;
        int rc;
        if (ASYNC) {
            rc = fcs_txq_send_async(Q, dst, 0x0800, payload, bsize);
        } else if (!DROPIN) {
            rc = fcs_txq_send(Q, dst, 0x0800, payload, bsize);
        } else {   /* src/linux/ether.c:257-265 with the drop-in ether_fcs */
            memcpy(frame, dst, 6);
            memcpy(frame + 6, MAC, 6);
            frame[12] = 0x08, frame[13] = 0x00;
            memcpy(frame + 14, payload, bsize);
            memset(frame + 14 + bsize, 0, fs - 14 - bsize);
            const uint32_t fcs = ether_fcs(frame, fs - 4);
            memcpy(frame + fs - 4, &fcs, 4);
            if (SOCK) {
                rc = (int)send(sock_tx, frame, fs, 0);
            } else {
                uint8_t *fp = frame;
                uint32_t sz = (uint32_t)fs;
                null_sink(NULL, &fp, &sz, &rc, 1);
            }
        }
        if (rc != (int)fs) atomic_fetch_add(&bad_results, 1);
    }
    return NULL;
}

int main(int argc, char **argv) {
    if (argc > 1) P = atoi(argv[1]);
    if (argc > 2) M = atoi(argv[2]);
    if (argc > 3) PAYLOAD = atoi(argv[3]);
    if (argc > 4) BATCH = atoi(argv[4]);
    if (argc > 5) FLUSH_US = atoi(argv[5]);
    if (argc > 6) SOCK = strcmp(argv[6], "sock") == 0;
    if (argc > 7) DROPIN = strcmp(argv[7], "dropin") == 0, ASYNC = strcmp(argv[7], "async") == 0;
    if (fcs_engine_init(1) < 0) {
        fprintf(stderr, "engine: %s\n", fcs_last_error());
        return 1;
    }
    pthread_t rd;
    if (SOCK) {
        int sv[2];
        if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv)) return perror("socketpair"), 1;
        int sz = 8 << 20;
        setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
        setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
        sock_tx = sv[0], sock_rx = sv[1];
        pthread_create(&rd, NULL, reader, NULL);
    }
    if (!DROPIN) {
        Q = fcs_txq_create(MAC, (uint32_t)BATCH, (uint32_t)FLUSH_US, SOCK ? fcs_txq_sink_fd : null_sink,
                           SOCK ? (void *)&sock_tx : NULL);
        if (!Q) return fprintf(stderr, "fcs_txq_create failed\n"), 1;
    } else {
        uint8_t warm[64] = {0};
        (void)ether_fcs(warm, 60);
    }
    pthread_t th[256];
    const double t0 = now();
    for (int t = 0; t < P; t++) pthread_create(&th[t], NULL, producer, (void *)(intptr_t)t);
    for (int t = 0; t < P; t++) pthread_join(th[t], NULL);
    if (Q) fcs_txq_flush(Q);
    const double t1 = now();
    uint64_t frames = 0, batches = 0, errors = 0, nr = 0, ng = 0, ns = 0, nb = 0, np_ = 0;
    if (Q) fcs_txq_stats(Q, &frames, &batches, &errors);
    if (Q) fcs_txq_timing(Q, &nr, &ng, &ns, &nb, &np_);
    if (SOCK) {
        while (atomic_load(&sunk_frames) < (unsigned long long)P * M && now() - t1 < 10) usleep(1000);
        shutdown(sock_tx, SHUT_RDWR);
        close(sock_tx);
        pthread_cancel(rd);
        pthread_join(rd, NULL);
    }
    const double dt = t1 - t0, nf = (double)P * M;
    printf("{\"mode\": \"%s\", \"sink\": \"%s\", \"producers\": %d, \"frames\": %.0f, \"payload\": %d, "
           "\"max_batch\": %d, \"flush_usec\": %d, \"s\": %.4f, \"Mframes_s\": %.4f, \"Gbit_s\": %.3f, "
           "\"mean_batch\": %.1f, \"bad_results\": %llu, \"sunk_frames\": %llu, \"queue_errors\": %llu, "
           "\"us_per_batch\": {\"ready\": %.1f, \"gpu\": %.1f, \"sink\": %.1f, \"busy\": %.1f, \"pickup\": %.1f, \"wall\": %.1f}}\n",
           DROPIN ? "dropin" : (ASYNC ? "async" : "txq"), SOCK ? "socketpair" : "null", P, nf, PAYLOAD, BATCH, FLUSH_US, dt,
           nf / dt / 1e6, (double)atomic_load(&sunk_bytes) * 8 / dt / 1e9, batches ? (double)frames / batches : 1.0,
           (unsigned long long)atomic_load(&bad_results), (unsigned long long)atomic_load(&sunk_frames),
           (unsigned long long)errors, batches ? nr / 1e3 / batches : 0.0, batches ? ng / 1e3 / batches : 0.0,
           batches ? ns / 1e3 / batches : 0.0, batches ? nb / 1e3 / batches : 0.0, batches ? np_ / 1e3 / batches : 0.0,
           batches ? dt * 1e6 / batches : 0.0);
    if (Q && errors) fprintf(stderr, "txq: %llu frames failed: %s\n", (unsigned long long)errors, fcs_txq_last_error(Q));
    if (Q) fcs_txq_destroy(Q);
    return (atomic_load(&bad_results) || errors) ? 2 : 0;
}
