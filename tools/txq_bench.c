/* txq_bench.c — rate of the batched TX call site (include/nstack_txq.h) against the per-frame
 * ether_send it replaces, on one GPU box, in one process.
 *
 *   tools/txq_bench [producers] [frames_per_producer] [payload|-1=random] [max_batch] [flush_usec]
 *                   [sink: null|sock] [mode: txq|async|dropin|reference|hostcrc] [host_max|-1]
 *                   [sync_host: 1|0]
 *
 * txq:       P producer threads call fcs_txq_send (ether_send semantics) into one queue; sync_host 0
 *            (fcs_txq_set_sync_host) makes their frames join batches and the GPU step instead of
 *            being sent by the callers themselves; host_max sets the GPU minimum of fire-and-forget
 *            batches (fcs_txq_set_host_max; -1 keeps the default, 0 sends every batch to the GPU).
 * async:     the same through fcs_txq_send_async (fire-and-forget; batches fill to max_batch).
 * reference: each producer runs the reference's ether_send body per frame
 *            (/root/reference/src/linux/ether.c:222-265): frame assembly in a stack buffer, the
 *            reference's OWN ether_fcs (src/ether_fcs.c compiled at its Makefile flags into
 *            oracle/_ref/libref_fcs.so by oracle/Makefile; override with NSTACK_REF_FCS_LIB), then
 *            the same sink for that one frame. A baseline leg: loaded with dlopen only in this
 *            mode, never linked into or called by the product.
 * dropin:    the same per-frame body with the library's drop-in ether_fcs() (GPU, one launch per
 *            frame) — today's ether_send with libnstack_fcs linked in place of ether_fcs.o.
 * hostcrc:   the same per-frame body with the library's host CRC (fcs_host_crc32) in the caller.
 * sink:      null = a counting sink; sock = an AF_UNIX datagram socketpair drained by a reader
 *            thread (the queue sends with one sendmmsg per batch, the per-frame modes with send()).
 * Prints one JSON line: frames/s, on-wire Gbit/s, mean batch, the queue's host/GPU batch split.
 * Build: gcc -O2 -pthread tools/txq_bench.c -Iinclude -Lnstack_amd -lnstack_fcs -ldl \
 *            -Wl,-rpath,'$ORIGIN/../nstack_amd' -o tools/txq_bench
 */
#define _GNU_SOURCE
#include <dlfcn.h>
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

enum { M_TXQ, M_ASYNC, M_DROPIN, M_REF, M_HOSTCRC };
static const char *MODE_NAME[] = {"txq", "async", "dropin", "reference", "hostcrc"};
static int P = 8, M = 20000, PAYLOAD = 1500, BATCH = 512, FLUSH_US = 0, SOCK = 0, MODE = M_TXQ;
static long long HOST_MAX = -1;
static int SYNC_HOST = 1;
static fcs_txq_t *Q;
static uint32_t (*ref_fcs)(const void *, size_t);   /* the reference's ether_fcs (reference mode) */
static int sock_tx = -1, sock_rx = -1;
static atomic_ullong sunk_frames, sunk_bytes, bad_results;
static atomic_int go;
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

/* src/linux/ether.c:222-265 for one frame, with the given FCS function */
static int per_frame_send(const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize,
                          uint32_t (*fcs_fn)(const void *, size_t)) {
    const size_t frame_size = 14 + (bsize > 56 ? bsize : 56) + 4;   /* :222-224 */
    uint8_t frame[frame_size] __attribute__((aligned));            /* :225 */
    if (frame_size > 1518) return -EMSGSIZE;                        /* :234-237 */
    memcpy(frame, dst, 6);                                          /* :257 */
    memcpy(frame + 6, MAC, 6);                                      /* :258 */
    frame[12] = (uint8_t)(proto >> 8), frame[13] = (uint8_t)proto;  /* :259 htons */
    memcpy(frame + 14, buf, bsize);                                 /* :260 */
    memset(frame + 14 + bsize, 0, frame_size - 14 - bsize);         /* :261 */
    const uint32_t fcs = fcs_fn(frame, frame_size - 4);             /* :262 */
    memcpy(frame + frame_size - 4, &fcs, 4);                        /* :263 */
    int rc;
    if (SOCK) {                                                     /* :265-269 */
        rc = (int)send(sock_tx, frame, frame_size, 0);
        if (rc < 0) rc = -errno;
    } else {
        uint8_t *fp = frame;
        uint32_t sz = (uint32_t)frame_size;
        null_sink(NULL, &fp, &sz, &rc, 1);
    }
    return rc;
}

static void *producer(void *arg) {
    const int t = (int)(intptr_t)arg;
    uint64_t s = 0x9E3779B97F4A7C15ull * (uint64_t)(t + 1);
    uint8_t payload[1500], dst[6] = {2, 0, 0, 0, 1, (uint8_t)t};
    for (int i = 0; i < 1500; i++) payload[i] = (uint8_t)(i * 31 + t);
    while (!atomic_load(&go)) ;
    for (int i = 0; i < M; i++) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        const size_t bsize = PAYLOAD >= 0 ? (size_t)PAYLOAD : (size_t)(s % 1501);
        const size_t fs = 14 + (bsize > 56 ? bsize : 56) + 4;
        int rc;
        switch (MODE) {
            case M_ASYNC: rc = fcs_txq_send_async(Q, dst, 0x0800, payload, bsize); break;
            case M_TXQ: rc = fcs_txq_send(Q, dst, 0x0800, payload, bsize); break;
            case M_DROPIN: rc = per_frame_send(dst, 0x0800, payload, bsize, ether_fcs); break;
            case M_REF: rc = per_frame_send(dst, 0x0800, payload, bsize, ref_fcs); break;
            default: rc = per_frame_send(dst, 0x0800, payload, bsize, fcs_host_crc32); break;
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
    if (argc > 7)
        for (int m = 0; m < 5; m++)
            if (!strcmp(argv[7], MODE_NAME[m])) MODE = m;
    if (argc > 8) HOST_MAX = atoll(argv[8]);
    if (argc > 9) SYNC_HOST = atoi(argv[9]) != 0;
    if (P < 1 || P > 256) return fprintf(stderr, "producers: 1..256\n"), 1;
    const int queue = MODE == M_TXQ || MODE == M_ASYNC;
    if (MODE == M_REF) {
        const char *path = getenv("NSTACK_REF_FCS_LIB");
        void *h = dlopen(path ? path : "oracle/_ref/libref_fcs.so", RTLD_NOW | RTLD_LOCAL);
        if (h) ref_fcs = (uint32_t (*)(const void *, size_t))dlsym(h, "ether_fcs");
        if (!ref_fcs) return fprintf(stderr, "reference ether_fcs: %s\n", dlerror()), 1;
        if (ref_fcs("123456789", 9) != 0xCBF43926u) return fprintf(stderr, "reference ether_fcs: wrong check value\n"), 1;
    } else if (MODE != M_HOSTCRC && fcs_engine_init(1) < 0) {
        fprintf(stderr, "engine: %s\n", fcs_last_error());
        if (!(MODE == M_TXQ && SYNC_HOST)) return 1;   /* synchronous callers send their own frames */
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
    long long host_max = -1;
    if (queue) {
        Q = fcs_txq_create(MAC, (uint32_t)BATCH, (uint32_t)FLUSH_US, SOCK ? fcs_txq_sink_fd : null_sink,
                           SOCK ? (void *)&sock_tx : NULL);
        if (!Q) return fprintf(stderr, "fcs_txq_create failed\n"), 1;
        const uint64_t dflt = fcs_txq_set_host_max(Q, 0);
        host_max = HOST_MAX >= 0 ? HOST_MAX : (long long)dflt;
        fcs_txq_set_host_max(Q, (uint64_t)host_max);
        /* warm the GPU step (first launch, mapped arrays) outside the timed region */
        const uint8_t d[6] = {2, 0, 0, 0, 0, 9}, pl[64] = {0};
        const uint64_t hm = fcs_txq_set_host_max(Q, 0);
        fcs_txq_set_sync_host(Q, 0);
        for (int i = 0; i < 4; i++) fcs_txq_send(Q, d, 0x0800, pl, sizeof pl);
        fcs_txq_set_host_max(Q, hm);
        fcs_txq_set_sync_host(Q, SYNC_HOST);
        while (SOCK && atomic_load(&sunk_frames) < 4) usleep(100);
    } else if (MODE == M_DROPIN) {
        uint8_t warm[64] = {0};
        (void)ether_fcs(warm, 60);
    }
    uint64_t f0 = 0, b0 = 0, sb0 = 0, sf0 = 0, gb0 = 0;
    if (Q) {
        fcs_txq_stats(Q, &f0, &b0, NULL);
        fcs_txq_small_batches(Q, &sb0, &sf0, &gb0);
    }
    const unsigned long long sunk0 = atomic_load(&sunk_frames), bytes0 = atomic_load(&sunk_bytes);
    pthread_t th[256];
    for (int t = 0; t < P; t++) pthread_create(&th[t], NULL, producer, (void *)(intptr_t)t);
    const double t0 = now();
    atomic_store(&go, 1);
    for (int t = 0; t < P; t++) pthread_join(th[t], NULL);
    if (Q) fcs_txq_flush(Q);
    const double t1 = now();
    uint64_t frames = 0, batches = 0, errors = 0, nr = 0, ng = 0, ns = 0, nb = 0, np_ = 0, sb = 0, sf = 0, gb = 0;
    if (Q) {
        fcs_txq_stats(Q, &frames, &batches, &errors);
        fcs_txq_timing(Q, &nr, &ng, &ns, &nb, &np_);
        fcs_txq_small_batches(Q, &sb, &sf, &gb);
        frames -= f0, batches -= b0, sb -= sb0, sf -= sf0, gb -= gb0;
    }
    const double nf = (double)P * M;
    if (SOCK) {
        while (atomic_load(&sunk_frames) - sunk0 < (unsigned long long)nf && now() - t1 < 10) usleep(1000);
        shutdown(sock_tx, SHUT_RDWR);
        close(sock_tx);
        pthread_cancel(rd);
        pthread_join(rd, NULL);
    }
    const double dt = t1 - t0;
    printf("{\"mode\": \"%s\", \"sink\": \"%s\", \"producers\": %d, \"frames\": %.0f, \"payload\": %d, "
           "\"max_batch\": %d, \"flush_usec\": %d, \"host_max\": %lld, \"sync_host\": %d, \"s\": %.4f, \"Mframes_s\": %.4f, "
           "\"us_per_frame_per_thread\": %.3f, \"Gbit_s\": %.3f, \"mean_batch\": %.1f, \"gpu_batches\": %llu, "
           "\"host_small_batches\": %llu, \"host_small_frames\": %llu, \"bad_results\": %llu, \"sunk_frames\": %llu, "
           "\"queue_errors\": %llu, \"us_per_batch\": {\"ready\": %.1f, \"fcs\": %.1f, \"sink\": %.1f, \"busy\": %.1f, "
           "\"pickup\": %.1f, \"wall\": %.1f}}\n",
           MODE_NAME[MODE], SOCK ? "socketpair" : "null", P, nf, PAYLOAD, queue ? BATCH : 1, FLUSH_US, host_max,
           queue ? SYNC_HOST : 1, dt,
           nf / dt / 1e6, dt * 1e6 * P / nf, (double)(atomic_load(&sunk_bytes) - bytes0) * 8 / dt / 1e9,
           batches ? (double)frames / batches : 1.0, (unsigned long long)gb, (unsigned long long)sb,
           (unsigned long long)sf, (unsigned long long)atomic_load(&bad_results),
           (unsigned long long)(atomic_load(&sunk_frames) - sunk0), (unsigned long long)errors,
           batches ? nr / 1e3 / batches : 0.0, batches ? ng / 1e3 / batches : 0.0, batches ? ns / 1e3 / batches : 0.0,
           batches ? nb / 1e3 / batches : 0.0, batches ? np_ / 1e3 / batches : 0.0, batches ? dt * 1e6 / batches : 0.0);
    if (Q && errors) fprintf(stderr, "txq: %llu frames failed: %s\n", (unsigned long long)errors, fcs_txq_last_error(Q));
    if (Q) fcs_txq_destroy(Q);
    return (atomic_load(&bad_results) || errors) ? 2 : 0;
}
