/* driver.c — runs every host-facing entry point of the product library, built with AddressSanitizer
 * + UBSan on its host code (tools/asan/Makefile), on a GPU box: the drop-in ether_fcs, the host
 * batch forms (pageable and pinned memory, packed / shuffled / fixed layouts, several pipeline
 * chunks, TX in place, RX verify), their argument errors, the TX queue (synchronous and
 * fire-and-forget producers, GPU step forced and default), the RX queue over a socketpair (GPU
 * check forced) and the Internet-checksum host batch. Results are checked against the library's
 * host CRC (fcs_host_crc32, pinned to the oracle by tests/test_host_crc.py) and the single-packet
 * checksum functions. Any sanitizer report aborts; a wrong result exits 1. Built with
 * -DDRIVER_FAULTS against the fault-hook build (libnstack_fcs_asan_faults.so, -DFCS_FAULT_HOOK) it
 * then drives the recovery paths: failed and timed-out drop-in attempts, host batch calls that
 * fail before their launch or give up with the kernel in flight (pipeline and small-batch stream
 * retired), a small batch held behind a busy kernel, and RX checks that give up after the launch.
 * Test tool only.
 *   tools/asan/run.sh   (ASAN_OPTIONS as there)
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
#include <sys/time.h>
#include <unistd.h>

#include "nstack_fcs.h"
#include "nstack_inet.h"
#include "nstack_rxq.h"
#include "nstack_txq.h"

static int failures;
#define CHECK(c, ...)                                                                  \
    do {                                                                               \
        if (!(c)) {                                                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                       \
            fprintf(stderr, __VA_ARGS__);                                              \
            fprintf(stderr, " (%s)\n", fcs_last_error());                              \
            failures++;                                                                \
        }                                                                              \
    } while (0)

static uint64_t rng_s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    rng_s ^= rng_s << 13, rng_s ^= rng_s >> 7, rng_s ^= rng_s << 17;
    return rng_s;
}
static void fill(uint8_t *p, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) p[i] = (uint8_t)(rnd() >> 24);
}

/* pinned memory when asked and available (fcs_host_alloc), else malloc; drop() frees either */
static uint8_t *take(uint64_t n, int want_pinned, int *pinned) {
    void *p = want_pinned ? fcs_host_alloc(n) : NULL;
    *pinned = p != NULL;
    return p ? p : malloc(n);
}
static void drop(void *p, int pinned) {
    if (pinned) fcs_host_free(p);
    else free(p);
}

static void dropin(void) {
    static uint8_t buf[200000];
    fill(buf, sizeof buf);
    const size_t lens[] = {0, 1, 3, 14, 60, 64, 127, 128, 129, 576, 1514, 1518, 1536, 1537, 2000, 3049,
                           9000, 65536, 100003, 200000};
    for (size_t k = 0; k < sizeof lens / sizeof lens[0]; k++) {
        const size_t off = lens[k] < 1000 ? (size_t)(rnd() % 1000) : 0;
        CHECK(ether_fcs(buf + off, lens[k]) == fcs_host_crc32(buf + off, lens[k]), "drop-in len %zu", lens[k]);
    }
}

/* variable-length frames: packed or shuffled offsets, pageable or pinned arena */
static void batch(uint64_t n, int pinned, int shuffled) {
    uint32_t *len = malloc(n * 4), *out = malloc(n * 4);
    uint64_t *off = malloc(n * 8), total = 0;
    for (uint64_t i = 0; i < n; i++) {
        len[i] = (uint32_t)(rnd() % 1600);
        off[i] = total;
        total += len[i] + (rnd() % 8);
    }
    if (shuffled)
        for (uint64_t i = n - 1; i > 0; i--) {
            const uint64_t j = rnd() % (i + 1), o = off[i];
            const uint32_t l = len[i];
            off[i] = off[j], len[i] = len[j], off[j] = o, len[j] = l;
        }
    uint8_t *arena = take(total + 8, pinned, &pinned);
    fill(arena, total + 8);
    CHECK(ether_fcs_batch_host(arena, total, off, len, out, n) == 0, "batch_host n %llu", (unsigned long long)n);
    for (uint64_t i = 0; i < n; i += 1 + n / 4096)
        CHECK(out[i] == fcs_host_crc32(arena + off[i], len[i]), "batch_host frame %llu", (unsigned long long)i);
    /* an out-of-range frame: -EINVAL and nothing written */
    memset(out, 0xAB, n * 4);
    off[n / 2] = total;
    len[n / 2] = 1;
    CHECK(ether_fcs_batch_host(arena, total, off, len, out, n) == -EINVAL, "out-of-range frame");
    CHECK(out[0] == 0xABABABABu && out[n - 1] == 0xABABABABu, "nothing written on -EINVAL");
    drop(arena, pinned);
    free(len), free(off), free(out);
}

static void fixed(uint64_t n, uint32_t L, uint64_t stride, int pinned) {
    const uint64_t bytes = (n - 1) * stride + L;
    uint8_t *base = take(bytes, pinned, &pinned);
    uint32_t *out = malloc(n * 4);
    fill(base, bytes);
    CHECK(ether_fcs_fixed_host(base, stride, L, n, out) == 0, "fixed_host %u", L);
    for (uint64_t i = 0; i < n; i += 1 + n / 4096)
        CHECK(out[i] == fcs_host_crc32(base + i * stride, L), "fixed_host frame %llu", (unsigned long long)i);
    CHECK(ether_fcs_fixed_host(base, L - 1, L, n, out) == -EINVAL, "stride < len");
    drop(base, pinned);
    free(out);
}

static void tx_and_verify(uint64_t n, int pinned) {
    const uint64_t stride = 1536, bytes = n * stride;
    uint8_t *base = take(bytes, pinned, &pinned);
    uint32_t *len = malloc(n * 4), *len4 = malloc(n * 4);
    uint64_t *off = malloc(n * 8);
    uint8_t *ok = malloc(n);
    fill(base, bytes);
    for (uint64_t i = 0; i < n; i++) {
        len[i] = 14 + (uint32_t)(rnd() % 1501);
        off[i] = i * stride;
        len4[i] = len[i] + 4;
    }
    CHECK(ether_fcs_tx_host(base, stride, len, n) == 0, "tx_host");
    for (uint64_t i = 0; i < n; i += 1 + n / 2048) {
        uint32_t c;
        memcpy(&c, base + i * stride + len[i], 4);
        CHECK(c == fcs_host_crc32(base + i * stride, len[i]), "tx_host frame %llu", (unsigned long long)i);
    }
    fill(base, bytes);
    CHECK(ether_fcs_tx_batch_host(base, bytes, off, len, n) == 0, "tx_batch_host");
    for (uint64_t i = 0; i < n; i += 1 + n / 2048) {
        uint32_t c;
        memcpy(&c, base + off[i] + len[i], 4);
        CHECK(c == fcs_host_crc32(base + off[i], len[i]), "tx_batch_host frame %llu", (unsigned long long)i);
    }
    /* every frame now carries its FCS: corrupt a few, verify */
    uint64_t want_bad = 0;
    for (uint64_t i = 0; i < n; i += 7) {
        base[off[i] + rnd() % len4[i]] ^= 0x20;
        want_bad++;
    }
    const int64_t bad = ether_fcs_verify_host(base, bytes, off, len4, ok, n);
    CHECK(bad == (int64_t)want_bad, "verify_host bad %lld want %llu", (long long)bad, (unsigned long long)want_bad);
    for (uint64_t i = 0; i < n; i++) CHECK(ok[i] == (i % 7 != 0), "verify_host ok[%llu]", (unsigned long long)i);
    CHECK(ether_fcs_tx_host(base, 16, len, n) == -EINVAL, "tx_host: frame + FCS past the stride");
    drop(base, pinned);
    free(len), free(len4), free(off), free(ok);
}

/* ---- TX queue ---- */
static atomic_ullong sunk, sunk_bad;
static void sink(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res, uint32_t n) {
    (void)ctx;
    for (uint32_t i = 0; i < n; i++) {
        if (fcs_host_crc32(frames[i], sizes[i]) != 0x2144DF1Cu) atomic_fetch_add(&sunk_bad, 1);
        res[i] = (int)sizes[i];
    }
    atomic_fetch_add(&sunk, n);
}
struct prod { fcs_txq_t *q; int async, frames, bad; };
static void *producer(void *a) {
    struct prod *p = a;
    const uint8_t dst[6] = {2, 0, 0, 0, 0, 2};
    uint8_t buf[1500];
    for (int i = 0; i < p->frames; i++) {
        const size_t n = (size_t)(i * 37 % 1501);
        memset(buf, i, n);
        const int r = p->async ? fcs_txq_send_async(p->q, dst, 0x0800, buf, n) : fcs_txq_send(p->q, dst, 0x0800, buf, n);
        if (r != (int)(14 + (n < 56 ? 56 : n) + 4)) p->bad++;   /* ether.c:222-224 */
    }
    return NULL;
}
static void txq_expect(int gpu_only, int no_host);
static void txq(int gpu_only) { txq_expect(gpu_only, 1); }
static void txq_expect(int gpu_only, int no_host) {
    const uint8_t mac[6] = {2, 0, 0, 0, 0, 1};
    fcs_txq_t *q = fcs_txq_create(mac, 256, 20, sink, NULL);
    CHECK(q != NULL, "txq create");
    if (!q) return;
    if (gpu_only) {
        fcs_txq_set_host_max(q, 0);
        fcs_txq_set_sync_host(q, 0);
    }
    atomic_store(&sunk, 0);
    atomic_store(&sunk_bad, 0);
    pthread_t th[6];
    struct prod p[6];
    for (int t = 0; t < 6; t++) {
        p[t] = (struct prod){q, t >= 4, 3000, 0};
        pthread_create(&th[t], NULL, producer, &p[t]);
    }
    for (int t = 0; t < 6; t++) {
        pthread_join(th[t], NULL);
        CHECK(p[t].bad == 0, "txq producer %d", t);
    }
    CHECK(fcs_txq_flush(q) == 0, "txq flush");
    uint64_t hb = 0, hf = 0;
    fcs_txq_fallbacks(q, &hb, &hf);
    CHECK(!no_host || hb == 0, "txq host answers %llu", (unsigned long long)hb);
    fcs_txq_destroy(q);
    CHECK(atomic_load(&sunk) == 18000 && atomic_load(&sunk_bad) == 0, "txq sunk %llu bad %llu",
          (unsigned long long)atomic_load(&sunk), (unsigned long long)atomic_load(&sunk_bad));
}

/* ---- RX queue over a socketpair, every batch checked on the GPU ---- */
static void rxq_expect(int no_host);
static void rxq(void) { rxq_expect(1); }
static void rxq_expect(int no_host) {
    int sv[2];
    CHECK(socketpair(AF_UNIX, SOCK_DGRAM, 0, sv) == 0, "socketpair");
    const int big = 8 << 20;
    setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    const uint8_t own[6] = {2, 0, 0, 0, 0, 9};
    uint8_t f[1518];
    int good = 0;
    for (int i = 0; i < 2000; i++) {
        const uint32_t L = 15 + (uint32_t)(rnd() % 1500);
        fill(f, L);
        f[6] = 2, f[7] = 0, f[8] = 0, f[9] = 0, f[10] = 0, f[11] = 7;
        const uint32_t c = fcs_host_crc32(f, L);
        memcpy(f + L, &c, 4);
        if (i % 9 == 3) f[rnd() % L] ^= 1;
        else good++;
        CHECK(send(sv[0], f, L + 4, 0) == (ssize_t)(L + 4), "send");
    }
    struct timeval tv = {0, 200000};
    setsockopt(sv[1], SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    fcs_rxq_t *q = fcs_rxq_create(sv[1], own, 64, FCS_RXQ_TRAILER);
    CHECK(q != NULL, "rxq create");
    if (!q) return;
    fcs_rxq_set_host_max(q, 0);
    struct fcs_ether_hdr h;
    uint8_t buf[1514];
    int got = 0, r;
    while ((r = fcs_rxq_receive(q, &h, buf, (size_t)(rnd() % 1515))) > 0) got++;
    uint64_t frames = 0, bad = 0, gpu = 0, hb = 0;
    fcs_rxq_stats(q, &frames, &bad, NULL, NULL, NULL);
    fcs_rxq_small_batches(q, NULL, NULL, &gpu);
    fcs_rxq_fallbacks(q, &hb, NULL);
    fcs_rxq_destroy(q);
    close(sv[0]), close(sv[1]);
    CHECK(got == good && frames == 2000 && bad == (uint64_t)(2000 - good) && gpu > 0 && (!no_host || hb == 0),
          "rxq got %d good %d bad %llu gpu %llu host %llu", got, good, (unsigned long long)bad,
          (unsigned long long)gpu, (unsigned long long)hb);
}

static void inet(void) {
    const uint64_t n = 20000;
    uint32_t *len = malloc(n * 4), *addr = malloc(n * 8);
    uint64_t *off = malloc(n * 8), total = 0;
    uint16_t *out = malloc(n * 2);
    for (uint64_t i = 0; i < n; i++) {
        len[i] = (uint32_t)(rnd() % 1600);
        off[i] = total;
        total += len[i];
        addr[2 * i] = (uint32_t)rnd();
        addr[2 * i + 1] = (uint32_t)rnd();
    }
    uint8_t *arena = malloc(total + 1);
    fill(arena, total + 1);
    for (int mode = 0; mode < 3; mode++) {
        CHECK(inet_csum_batch_host(mode, arena, total, off, len, mode ? addr : NULL, out, n) == 0, "inet mode %d", mode);
        for (uint64_t i = 0; i < n; i += 97) {
            const uint8_t *p = arena + off[i];
            const uint16_t w = mode == 0   ? inet_ip_checksum(p, len[i])
                               : mode == 1 ? inet_tcp_checksum(addr[2 * i], addr[2 * i + 1], p, len[i])
                                           : inet_udp_checksum(p, len[i], addr[2 * i], addr[2 * i + 1]);
            CHECK(out[i] == w, "inet mode %d packet %llu", mode, (unsigned long long)i);
        }
    }
    free(len), free(addr), free(off), free(out), free(arena);
}

#ifdef DRIVER_FAULTS
void fcs_debug_fail_next(int attempts);
void fcs_debug_timeout_next(int attempts);
void fcs_debug_fail_batches(int skip, int calls);
void fcs_debug_late_batches(int skip, int calls);
void fcs_debug_hold_small(const uint32_t *word);
uint32_t fcs_debug_retired(void);

static void *release_word(void *w) {
    usleep(300000);
    __atomic_store_n((uint32_t *)w, 1u, __ATOMIC_SEQ_CST);
    return NULL;
}

static void faults(void) {
    static uint8_t buf[4000];
    fill(buf, sizeof buf);
    /* drop-in: one failed attempt (retried on a fresh lane), two (host answer), a timeout */
    fcs_debug_fail_next(1);
    CHECK(ether_fcs(buf, 1514) == fcs_host_crc32(buf, 1514), "drop-in after one failure");
    fcs_debug_fail_next(2);
    CHECK(ether_fcs(buf, 1000) == fcs_host_crc32(buf, 1000), "drop-in after two failures");
    fcs_debug_timeout_next(1);
    CHECK(ether_fcs(buf, 3000) == fcs_host_crc32(buf, 3000), "drop-in after a timeout");
    /* host batches: failure before the launch, then with the kernel in flight (pipeline retired) */
    const uint32_t r0 = fcs_debug_retired();
    fcs_debug_fail_batches(0, 1);
    batch(5000, 0, 0);
    fcs_debug_late_batches(0, 1);
    batch(400000, 0, 0);
    fcs_debug_late_batches(1, 1);   /* the second call of this pair */
    fixed(300000, 1518, 1536, 1);
    fixed(300000, 1518, 1536, 0);
    batch(20000, 0, 1);             /* healthy again, on a fresh pipeline */
    /* small TX batches in pinned memory: late failures retire the small-batch stream */
    for (int k = 0; k < 3; k++) {
        fcs_debug_late_batches(k, 1);
        tx_and_verify(40, 1);
        tx_and_verify(40, 1);
    }
    /* a small batch queued behind a kernel that stays busy until a pinned word is set */
    uint32_t *word = (uint32_t *)fcs_host_alloc(64);
    CHECK(word != NULL, "pinned word");
    if (word) {
        memset(word, 0, 64);
        pthread_t rel;
        pthread_create(&rel, NULL, release_word, word);
        fcs_debug_hold_small(word);
        fcs_debug_late_batches(0, 1);
        tx_and_verify(8, 1);        /* answered by the host while the held kernel runs */
        tx_and_verify(8, 1);        /* the next one on a fresh stream */
        pthread_join(rel, NULL);
    }
    CHECK(fcs_debug_retired() > r0, "a pipeline or stream was retired");
    /* RX: pipelined checks that give up after their launch */
    fcs_debug_late_batches(2, 3);
    rxq_expect(0);
    /* TX queue with the GPU step forced and batch failures */
    fcs_debug_fail_batches(3, 2);
    fcs_debug_late_batches(6, 2);
    txq_expect(1, 0);
    if (word) fcs_host_free(word);
}
#endif

int main(void) {
    dropin();
    batch(5000, 0, 0);
    batch(5000, 1, 0);
    batch(20000, 0, 1);
    batch(400000, 0, 0);   /* ~330 MB: three pipeline chunks */
    fixed(300000, 1518, 1518, 0);
    fixed(300000, 1518, 1536, 1);
    fixed(5000, 9000, 9000, 0);
    tx_and_verify(3000, 0);
    tx_and_verify(3000, 1);
    tx_and_verify(60000, 1);
    txq(0);
    txq(1);
    rxq();
    inet();
    uint64_t fb = fcs_engine_host_fallbacks(), hb = fcs_engine_host_batches();
    CHECK(fb == 0 && hb == 0, "host answers: drop-in %llu, batches %llu", (unsigned long long)fb, (unsigned long long)hb);
#ifdef DRIVER_FAULTS
    faults();
    fb = fcs_engine_host_fallbacks(), hb = fcs_engine_host_batches();
    CHECK(fb >= 1 && hb >= 3, "host answers under faults: drop-in %llu, batches %llu", (unsigned long long)fb,
          (unsigned long long)hb);
#endif
    fcs_engine_fini();
    printf("asan driver: %s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
