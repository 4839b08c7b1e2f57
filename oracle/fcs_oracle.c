/*
 * oracle/fcs_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * The product library (nstack_amd/libnstack_fcs.so) never loads or calls it. The product's own
 * host CRC (nstack_amd/csrc/fcs_host_crc.cpp, slice-by-16 with tables derived at run time) is a
 * separate implementation used only when a GPU step fails (the drop-in after its retry, the TX/RX
 * queues per batch), counted, and asserted unused by the GPU suite.
 *
 * What it restates:
 *   ether_fcs()  /root/reference/src/ether_fcs.c:4-19
 *     - a 16-entry nibble table for the reflected CRC-32 polynomial 0xEDB88320 with the
 *       register complement folded into the table (table[i] = T16[15 - i] ^ 0xF0000000,
 *       src/ether_fcs.c:7-10), register initialised to 0 (:11), two table steps per byte,
 *       low nibble first (:13-16), no final XOR (:18).
 *     The table here is DERIVED from the polynomial at first use instead of being written
 *     out, and oracle_selfcheck() verifies the derivation against the known answers in
 *     SURVEY.md §8c ("123456789" -> 0xCBF43926, residue 0x2144DF1C).
 *   A slice-by-8 variant (oracle_crc32_fast) computes the same function (CRC-32/ISO-HDLC)
 *   about 10x faster; it is used to check multi-GiB GPU runs, never as the baseline.
 *
 * Pinning: tests/test_oracle.py checks both against the golden fixtures in tests/golden/
 * (generated from the reference's own src/ether_fcs.c compiled by oracle/Makefile into
 * oracle/_ref/, see tests/golden/make_golden.py) and against zlib.crc32.
 *
 * Data generators (shared with the GPU tests / bench so inputs can be re-created on CPU):
 *   oracle_xorshift64_fill  — the SURVEY §8c/§8d dataset (seed 42, s^=s<<13; s^=s>>7;
 *                             s^=s<<17; byte = low 8 bits of s after each step).
 *   oracle_splitmix_fill    — counter-based bytes: 8-byte word w at byte offset 8*w is
 *                             splitmix64(seed + w) little-endian; matches the device
 *                             generator fcs_fill_splitmix64 in the product library.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <time.h>
#include <pthread.h>

#define POLY_REFLECTED 0xEDB88320u

static uint32_t nib_table[16];   /* complement-folded nibble table (src/ether_fcs.c:7-10) */
static uint32_t slice8[8][256];  /* standard reflected slice-by-8 tables */
static int tables_ready;

static uint32_t reflected_shift(uint32_t r, int bits)
{
    for (int b = 0; b < bits; b++)
        r = (r >> 1) ^ ((r & 1u) ? POLY_REFLECTED : 0u);
    return r;
}

static void build_tables(void)
{
    if (tables_ready)
        return;
    /* T16[k]: four reflected shift steps of k; folded: table[i] = T16[15-i] ^ 0xF0000000 */
    for (int i = 0; i < 16; i++)
        nib_table[i] = reflected_shift((uint32_t)(15 - i), 4) ^ 0xF0000000u;
    for (int b = 0; b < 256; b++)
        slice8[0][b] = reflected_shift((uint32_t)b, 8);
    for (int k = 1; k < 8; k++)
        for (int b = 0; b < 256; b++)
            slice8[k][b] = (slice8[k - 1][b] >> 8) ^ slice8[0][slice8[k - 1][b] & 0xFF];
    tables_ready = 1;
}

/* Restatement of ether_fcs (src/ether_fcs.c:4-19): register 0, folded table, 2 nibbles/byte. */
uint32_t oracle_ether_fcs(const void *data, size_t bsize)
{
    const uint8_t *p = (const uint8_t *) data;
    uint32_t r = 0;
    if (!tables_ready)
        build_tables();
    for (size_t i = 0; i < bsize; i++) {
        r = (r >> 4) ^ nib_table[(r ^ p[i]) & 0x0F];        /* low nibble  (:14) */
        r = (r >> 4) ^ nib_table[(r ^ (p[i] >> 4)) & 0x0F]; /* high nibble (:15) */
    }
    return r;
}

/* Same function, slice-by-8 over the standard (non-folded) register: ~r in, ~r out. */
uint32_t oracle_crc32_fast_from(uint32_t r, const void *data, size_t n);
uint32_t oracle_crc32_fast(const void *data, size_t n)
{
    return oracle_crc32_fast_from(0xFFFFFFFFu, data, n);
}

/* The slice-by-8 register walk from register r (the standard, non-complemented register). */
uint32_t oracle_crc32_fast_from(uint32_t r, const void *data, size_t n)
{
    const uint8_t *p = (const uint8_t *) data;
    if (!tables_ready)
        build_tables();
    while (n && ((uintptr_t) p & 7)) {
        r = (r >> 8) ^ slice8[0][(r ^ *p++) & 0xFF];
        n--;
    }
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= r;
        r = slice8[7][lo & 0xFF] ^ slice8[6][(lo >> 8) & 0xFF] ^
            slice8[5][(lo >> 16) & 0xFF] ^ slice8[4][lo >> 24] ^
            slice8[3][hi & 0xFF] ^ slice8[2][(hi >> 8) & 0xFF] ^
            slice8[1][(hi >> 16) & 0xFF] ^ slice8[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--)
        r = (r >> 8) ^ slice8[0][(r ^ *p++) & 0xFF];
    return ~r;
}

/* Batch helpers. fast=0 -> nibble restatement, fast=1 -> slice-by-8. */
void oracle_fcs_batch(const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                      uint32_t *out, size_t n, int fast)
{
    for (size_t i = 0; i < n; i++)
        out[i] = fast ? oracle_crc32_fast(arena + off[i], len[i])
                      : oracle_ether_fcs(arena + off[i], len[i]);
}

struct fixed_job {
    const uint8_t *base;
    size_t stride, n;
    uint32_t len;
    uint32_t *out;
    int fast;
};

static void *fixed_worker(void *arg)
{
    struct fixed_job *j = (struct fixed_job *) arg;
    for (size_t i = 0; i < j->n; i++)
        j->out[i] = j->fast ? oracle_crc32_fast(j->base + i * j->stride, j->len)
                            : oracle_ether_fcs(j->base + i * j->stride, j->len);
    return NULL;
}

/* Fixed-stride frames, optionally over nthreads host threads (contiguous shards). */
void oracle_fcs_fixed(const uint8_t *base, size_t stride, uint32_t len, size_t n,
                      uint32_t *out, int fast, int nthreads)
{
    if (!tables_ready)
        build_tables();
    if (nthreads <= 1) {
        struct fixed_job j = {base, stride, n, len, out, fast};
        fixed_worker(&j);
        return;
    }
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct fixed_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        size_t lo = n * (size_t) t / (size_t) nthreads;
        size_t hi = n * (size_t)(t + 1) / (size_t) nthreads;
        jobs[t] = (struct fixed_job){base + lo * stride, stride, hi - lo, len, out + lo, fast};
        pthread_create(&th[t], NULL, fixed_worker, &jobs[t]);
    }
    for (int t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
}

/* Wall-clock seconds of oracle_fcs_fixed (for bench.py's cpu_baseline leg). */
double oracle_time_fixed(const uint8_t *base, size_t stride, uint32_t len, size_t n,
                         uint32_t *out, int fast, int nthreads)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oracle_fcs_fixed(base, stride, len, n, out, fast, nthreads);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Wall-clock seconds of `n` calls fcs(base + i*stride, len) of an ether_fcs-shaped function: the
 * reference's own compiled src/ether_fcs.c (oracle/_ref) for bench.py's cpu_baseline leg, called
 * once per frame exactly as ether_send calls it (src/linux/ether.c:262). */
typedef uint32_t (*fcs_fn)(const void *, size_t);
double oracle_time_calls(fcs_fn fcs, const uint8_t *base, size_t stride, uint32_t len, size_t n, uint32_t *out)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (size_t i = 0; i < n; i++) out[i] = fcs(base + i * stride, len);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* SURVEY §8c dataset: xorshift64, one output byte per step; *state carries across calls. */
void oracle_xorshift64_fill(uint8_t *buf, size_t n, uint64_t *state)
{
    uint64_t s = *state;
    for (size_t i = 0; i < n; i++) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        buf[i] = (uint8_t) s;
    }
    *state = s;
}

static uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* Bytes [byte_offset, byte_offset + n) of the counter-based stream for `seed`. */
void oracle_splitmix_fill(uint8_t *buf, size_t n, uint64_t seed, uint64_t byte_offset)
{
    for (size_t i = 0; i < n; i++) {
        uint64_t pos = byte_offset + i;
        uint64_t w = splitmix64(seed + (pos >> 3));
        buf[i] = (uint8_t)(w >> (8 * (pos & 7)));
    }
}

/* Bytes [byte_offset, byte_offset + n) of the same stream, one splitmix64 per 8-byte word. */
static void splitmix_fill_words(uint8_t *buf, size_t n, uint64_t seed, uint64_t byte_offset)
{
    size_t i = 0;
    while (i < n && ((byte_offset + i) & 7)) {
        uint64_t pos = byte_offset + i;
        buf[i++] = (uint8_t)(splitmix64(seed + (pos >> 3)) >> (8 * (pos & 7)));
    }
    for (; i + 8 <= n; i += 8) {
        uint64_t w = splitmix64(seed + ((byte_offset + i) >> 3));
        memcpy(buf + i, &w, 8);   /* little-endian host: byte k of the word is bits 8k..8k+7 */
    }
    for (; i < n; i++) {
        uint64_t pos = byte_offset + i;
        buf[i] = (uint8_t)(splitmix64(seed + (pos >> 3)) >> (8 * (pos & 7)));
    }
}

/* Digest of a whole splitmix batch without materialising it: frame i is the stream's bytes
 * [off_i, off_i + len_i) (off == NULL: i * stride, len == NULL: flen); the XOR and the 64-bit sum of
 * every frame's CRC (slice-by-8), over nthreads host threads. For checking full BASELINE-size GPU
 * launches (tests/test_gpu_parity.py): 64 M x 1518 B, 128 M IMIX frames, 16 M x 9000 B. */
struct digest_job {
    uint64_t seed, stride, i0, i1;
    const uint64_t *off;
    const uint32_t *len;
    uint32_t flen;
    uint32_t x;
    uint64_t sum;
};

static void *digest_worker(void *arg)
{
    struct digest_job *j = (struct digest_job *) arg;
    uint8_t buf[65536 + 16];
    uint32_t x = 0;
    uint64_t sum = 0;
    for (uint64_t i = j->i0; i < j->i1; i++) {
        const uint64_t o = j->off ? j->off[i] : i * j->stride;
        const uint32_t L = j->len ? j->len[i] : j->flen;
        uint32_t c;
        if (L <= 65536) {
            splitmix_fill_words(buf, L, j->seed, o);
            c = oracle_crc32_fast(buf, L);
        } else {   /* longer frames: in pieces, the register carried (~c in, ~c out) */
            c = 0;   /* the CRC so far; its register is ~c */
            for (uint64_t k = 0; k < L; k += 65536) {
                size_t m = L - k < 65536 ? (size_t)(L - k) : 65536;
                splitmix_fill_words(buf, m, j->seed, o + k);
                c = oracle_crc32_fast_from(~c, buf, m);
            }
        }
        x ^= c;
        sum += c;
    }
    j->x = x;
    j->sum = sum;
    return NULL;
}

void oracle_splitmix_digest(uint64_t seed, const uint64_t *off, const uint32_t *len, uint64_t stride,
                            uint32_t flen, uint64_t n, int nthreads, uint32_t *xor_out, uint64_t *sum_out)
{
    if (!tables_ready)
        build_tables();
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct digest_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct digest_job){seed, stride, n * (uint64_t) t / (uint64_t) nthreads,
                                      n * (uint64_t)(t + 1) / (uint64_t) nthreads, off, len, flen, 0, 0};
        pthread_create(&th[t], NULL, digest_worker, &jobs[t]);
    }
    uint32_t x = 0;
    uint64_t sum = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        x ^= jobs[t].x;
        sum += jobs[t].sum;
    }
    *xor_out = x;
    *sum_out = sum;
}

/* 0 on success; checks the derived tables against SURVEY §8c known answers. */
int oracle_selfcheck(void)
{
    static const char kv[] = "123456789";
    uint8_t buf[64];
    if (oracle_ether_fcs(kv, 9) != 0xCBF43926u || oracle_crc32_fast(kv, 9) != 0xCBF43926u)
        return 1;
    if (oracle_ether_fcs(kv, 0) != 0)
        return 2;
    for (int n = 0; n < 60; n++) {
        for (int i = 0; i < n; i++)
            buf[i] = (uint8_t)(i * 37 + 11);
        uint32_t c = oracle_ether_fcs(buf, (size_t) n);
        memcpy(buf + n, &c, 4);
        if (oracle_ether_fcs(buf, (size_t) n + 4) != 0x2144DF1Cu)
            return 3;
    }
    return 0;
}
