/* rxq_bench.c — rate of the batched RX call site (include/nstack_rxq.h) on one GPU box, beside the
 * reference's per-frame ether_receive.
 *
 *   tools/rxq_bench [frames] [payload] [max_batch] [trailer: 0|1] [mode: queue|reference] [host_max|-1]
 *
 * A sender thread pushes `frames` ether_send-built frames (their FCS computed once by the engine,
 * ether_fcs_tx_host) through an AF_UNIX datagram socketpair with sendmmsg; the main thread takes
 * them out one per call with fcs_rxq_receive, which refills with recvmmsg and (trailer=1)
 * verifies every batch (on the GPU above the GPU minimum host_max, fcs_rxq_set_host_max; -1 keeps
 * the default, 0 sends every batch to the GPU). trailer=0 is the same path without any check.
 * reference: ether_receive's body per call (/root/reference/src/linux/ether.c:193-211): one
 * recvfrom into a 1514-B stack buffer, the own-MAC echo test, the header and payload copies; it
 * checks no FCS (run it with trailer=0). Prints one JSON line: frames/s, Gbit/s of frame bytes,
 * mean batch, and the counters.
 * Build: gcc -O2 -pthread tools/rxq_bench.c -Iinclude -Lnstack_amd -lnstack_fcs \
 *            -Wl,-rpath,'$ORIGIN/../nstack_amd' -o tools/rxq_bench
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "nstack_fcs.h"
#include "nstack_rxq.h"

static int N = 200000, PAYLOAD = 1500, BATCH = 64, TRAILER = 1, REF = 0;
static long long HOST_MAX = -1;
static int sv[2];
static uint8_t *frames;
static uint32_t flen;
enum { POOL = 1024 };

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *sender(void *arg) {
    (void)arg;
    struct mmsghdr m[64];
    struct iovec iov[64];
    int sent = 0;
    while (sent < N) {
        int k = N - sent < 64 ? N - sent : 64;
        for (int i = 0; i < k; i++) {
            iov[i].iov_base = frames + (size_t)((sent + i) % POOL) * 1536;
            iov[i].iov_len = flen;
            memset(&m[i], 0, sizeof m[i]);
            m[i].msg_hdr.msg_iov = &iov[i];
            m[i].msg_hdr.msg_iovlen = 1;
        }
        int r = sendmmsg(sv[0], m, k, 0);
        if (r > 0) sent += r;
    }
    return NULL;
}

int main(int argc, char **argv) {
    if (argc > 1) N = atoi(argv[1]);
    if (argc > 2) PAYLOAD = atoi(argv[2]);
    if (argc > 3) BATCH = atoi(argv[3]);
    if (argc > 4) TRAILER = atoi(argv[4]);
    if (argc > 5) REF = strcmp(argv[5], "reference") == 0;
    if (argc > 6) HOST_MAX = atoll(argv[6]);
    if (REF && TRAILER) return fprintf(stderr, "reference mode receives frames without a trailer\n"), 1;
    if (fcs_engine_init(1) < 0 && (TRAILER || !REF)) return fprintf(stderr, "engine: %s\n", fcs_last_error()), 1;
    const uint8_t own[6] = {2, 0, 0, 0, 0, 1}, peer[6] = {2, 0, 0, 0, 0, 2};
    const uint32_t body = 14 + (PAYLOAD > 56 ? PAYLOAD : 56);
    flen = body + (TRAILER ? 4 : 0);
    frames = fcs_host_alloc((size_t)POOL * 1536);
    if (!frames) frames = malloc((size_t)POOL * 1536);
    uint32_t *cov = malloc(POOL * 4);
    for (int i = 0; i < POOL; i++) {
        uint8_t *f = frames + (size_t)i * 1536;
        memset(f, 0, 1536);
        memcpy(f, own, 6);
        memcpy(f + 6, peer, 6);
        f[12] = 0x08, f[13] = 0x00;
        for (int b = 0; b < PAYLOAD; b++) f[14 + b] = (uint8_t)(b * 7 + i);
        cov[i] = body;
    }
    if (TRAILER && ether_fcs_tx_host(frames, 1536, cov, POOL)) return fprintf(stderr, "%s\n", fcs_last_error()), 1;
    if (socketpair(AF_UNIX, SOCK_DGRAM, 0, sv)) return perror("socketpair"), 1;
    int sz = 16 << 20;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &sz, sizeof sz);
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &sz, sizeof sz);
    fcs_rxq_t *q = REF ? NULL : fcs_rxq_create(sv[1], own, BATCH, TRAILER ? FCS_RXQ_TRAILER : 0);
    if (!REF && !q) return fprintf(stderr, "fcs_rxq_create failed\n"), 1;
    long long host_max = -1;
    if (q) {
        const uint64_t dflt = fcs_rxq_set_host_max(q, 0);
        host_max = HOST_MAX >= 0 ? HOST_MAX : (long long)dflt;
        fcs_rxq_set_host_max(q, (uint64_t)host_max);
    }
    struct fcs_ether_hdr h;
    static uint8_t buf[2048];
    (void)fcs_rxq_receive;
    pthread_t th;
    const double t0 = now();
    pthread_create(&th, NULL, sender, NULL);
    int got = 0, errs = 0;
    while (got < N) {
        int r;
        if (REF) {   /* src/linux/ether.c:193-211 */
            uint8_t frame[1514] __attribute__((aligned));
            do {
                r = (int)recvfrom(sv[1], frame, sizeof frame, 0, NULL, NULL);
                if (r == -1) break;
            } while (!memcmp(frame + 6, own, 6));
            if (r > 0) {
                memcpy(h.h_dst, frame, 6);
                memcpy(h.h_src, frame + 6, 6);
                h.h_proto = (uint16_t)((frame[12] << 8) | frame[13]);
                r -= 14;
                memcpy(buf, frame + 14, (size_t)r < sizeof buf ? (size_t)r : sizeof buf);
                r = r > 0 ? r : 1;
            }
        } else {
            r = fcs_rxq_receive(q, &h, buf, sizeof buf);
        }
        if (r > 0) got++;
        else if (r < 0 && ++errs > 10) return fprintf(stderr, "receive: %d %s\n", r, fcs_last_error()), 1;
    }
    const double t1 = now();
    pthread_join(th, NULL);
    uint64_t fr = N, bad = 0, echo = 0, drop = 0, batches = N, sb = 0, sf = 0, gb = 0;
    if (q) {
        fcs_rxq_stats(q, &fr, &bad, &echo, &drop, &batches);
        fcs_rxq_small_batches(q, &sb, &sf, &gb);
    }
    printf("{\"mode\": \"%s\", \"trailer\": %d, \"frames\": %d, \"payload\": %d, \"max_batch\": %d, "
           "\"host_max\": %lld, \"s\": %.4f, \"Mframes_s\": %.4f, \"Gbit_s\": %.3f, \"mean_batch\": %.1f, "
           "\"host_batches\": %llu, \"gpu_batches\": %llu, \"bad_fcs\": %llu, \"echoes\": %llu, \"dropped\": %llu}\n",
           REF ? "reference" : "queue", TRAILER, N, PAYLOAD, REF ? 1 : BATCH, host_max, t1 - t0, N / (t1 - t0) / 1e6,
           (double)N * flen * 8 / (t1 - t0) / 1e9, batches ? (double)fr / batches : 0.0, (unsigned long long)sb,
           (unsigned long long)gb, (unsigned long long)bad, (unsigned long long)echo, (unsigned long long)drop);
    if (q) fcs_rxq_destroy(q);
    fcs_host_free(frames);
    return bad ? 2 : 0;
}
