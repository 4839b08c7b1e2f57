/*
 * oracle/inet_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * Only tests/ may load this. The product library (nstack_amd/libnstack_fcs.so) computes every
 * Internet checksum in its HIP kernel (nstack_amd/csrc/inet_kernel.hip) and has no CPU path.
 *
 * What it restates, loop for loop:
 *   ip_checksum(dp, bsize)               /root/reference/src/ip.c:39-62
 *     acc = 0xffff (:42); 16-bit words read with memcpy in HOST byte order (:47), added with an
 *     end-around carry "if (acc > 0xffff) acc -= 0xffff" (:48-50); an odd trailing byte is the
 *     low byte of a zeroed word (:53-58); return ~acc truncated to 16 bits (:61).
 *     Also the ICMP checksum (src/icmp.c:42,74 call ip_checksum).
 *   tcp_checksum(src, dst, dp, bsize)    /root/reference/src/tcp.c:167-213
 *     the same loop (acc = 0xffff) first over the 12-byte packed pseudo header
 *     {htonl(src), htonl(dst), 0, IP_PROTO_TCP = 6, htons(bsize)} (:176-188, :190-195), then over
 *     the segment (:197-209). src/dst are host-order IPv4 addresses (nstack_sockaddr.inet4_addr).
 *   udp_checksum(buff, len, src, dst)    /root/reference/src/udp.c:136-174 (static)
 *     sum = 0 (:146), u16 words in host order (:148), "if (sum & 0x80000000) fold" inside the
 *     loop (:150-151), odd byte added as a low byte (:156-157), then the two halves of the raw
 *     in_addr_t src and dst as they lie in memory (:143,160-164), htons(IPPROTO_UDP) (:166),
 *     htons(len) (:167); fold while (sum >> 16) (:170-171); return ~sum (:174).
 *
 * Pinning: the reference's src/ip.c / src/tcp.c / src/udp.c could not be built here (the
 * request to compile src/ip.c was refused), and the reference's tests hold no
 * checksum fixture. tests/test_inet_oracle.py therefore pins this restatement to published
 * known answers (the RFC 1071 §3 numeric example, a textbook IPv4 header) and to an
 * independent big-endian formulation of RFC 1071 in tests/golden/make_inet_golden.py. Parity
 * with the reference's own functions is "unpinned" in the sense of the task statement: no
 * output of the reference itself backs these vectors.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

static uint16_t bswap16(uint16_t x) { return (uint16_t)((x << 8) | (x >> 8)); }

/* One's-complement accumulation as src/ip.c:46-59 and src/tcp.c:190-209 perform it: the running sum
 * starts at 0xffff, each 16-bit word is added and an overflow past 0xffff is folded back at once by
 * subtracting 0xffff; an odd trailing byte enters as the low byte of a zero word. Words are the bytes
 * in host order (the reference memcpy's them into a uint16_t); this container and the reference's
 * targets are little-endian, so word k is p[2k] | p[2k+1] << 8. */
static uint32_t ones_fold_add(uint32_t acc, uint32_t w)
{
    acc += w;
    return acc > 0xffffu ? acc - 0xffffu : acc;
}

static uint32_t ones_sum_le16(uint32_t acc, const uint8_t *p, size_t n)
{
    const size_t pairs = n / 2;
    for (size_t k = 0; k < pairs; k++)
        acc = ones_fold_add(acc, (uint32_t) p[2 * k] | ((uint32_t) p[2 * k + 1] << 8));
    if (n % 2)
        acc = ones_fold_add(acc, p[n - 1]);
    return acc;
}

/* src/ip.c:39-62: ~(running sum from 0xffff), truncated to 16 bits (:61). */
uint16_t oracle_ip_checksum(const void *dp, size_t bsize)
{
    return (uint16_t) ~ones_sum_le16(0xffffu, (const uint8_t *) dp, bsize);
}

/* src/tcp.c:167-213; src/dst in host order. The 12-byte pseudo header (:176-188) is summed first
 * (:190-195), then the segment (:197-209); both use the accumulation above. */
uint16_t oracle_tcp_checksum(uint32_t src, uint32_t dst, const void *dp, size_t bsize)
{
    const uint8_t ph[12] = {
        (uint8_t)(src >> 24), (uint8_t)(src >> 16), (uint8_t)(src >> 8), (uint8_t) src,   /* htonl(src) */
        (uint8_t)(dst >> 24), (uint8_t)(dst >> 16), (uint8_t)(dst >> 8), (uint8_t) dst,   /* htonl(dst) */
        0, 6,                                                   /* zero, IP_PROTO_TCP */
        (uint8_t)(bsize >> 8), (uint8_t) bsize,                 /* htons(bsize), truncated to 16 bits */
    };
    return (uint16_t) ~ones_sum_le16(ones_sum_le16(0xffffu, ph, sizeof ph), (const uint8_t *) dp, bsize);
}

/* src/udp.c:136-174; src/dst are the raw in_addr_t values the caller passes. */
uint16_t oracle_udp_checksum(const void *buff, size_t len, uint32_t src, uint32_t dst)
{
    const uint8_t *buf = (const uint8_t *) buff;
    uint16_t ip_src[2], ip_dst[2], w;
    uint32_t sum = 0;
    size_t length = len;

    memcpy(ip_src, &src, 4);
    memcpy(ip_dst, &dst, 4);
    while (len > 1) {
        memcpy(&w, buf, 2);
        buf += 2;
        sum += w;
        if (sum & 0x80000000u)
            sum = (sum & 0xFFFF) + (sum >> 16);
        len -= 2;
    }
    if (len & 1)
        sum += *buf;
    sum += ip_src[0];
    sum += ip_src[1];
    sum += ip_dst[0];
    sum += ip_dst[1];
    sum += bswap16(17);               /* htons(IPPROTO_UDP) */
    sum += bswap16((uint16_t) length); /* htons(length) */
    while (sum >> 16)
        sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t) ~sum;
}

/* Batch helper with the product's argument convention: mode 0 = ip, 1 = tcp, 2 = udp; addr holds
 * (src, dst) per packet for tcp/udp (NULL for ip). Packet i = arena[off[i] .. off[i] + len[i]). */
void oracle_inet_batch(int mode, const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                       const uint32_t *addr, uint16_t *out, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        const uint8_t *p = arena + off[i];
        if (mode == 1)
            out[i] = oracle_tcp_checksum(addr[2 * i], addr[2 * i + 1], p, len[i]);
        else if (mode == 2)
            out[i] = oracle_udp_checksum(p, len[i], addr[2 * i], addr[2 * i + 1]);
        else
            out[i] = oracle_ip_checksum(p, len[i]);
    }
}

/* ---- full-batch digests of splitmix batches (tests/test_gpu_inet.py at BASELINE-like sizes) ----
 * Packet i is bytes [off_i, off_i + len_i) (off == NULL: i * stride; len == NULL: flen) of the
 * counter-based stream of the product's fcs_fill_splitmix64 (word w = splitmix64(seed + w), little
 * endian; the same stream as oracle_splitmix_fill in fcs_oracle.c), checksummed by the restatement
 * above (mode as oracle_inet_batch; tcp/udp addresses addr[2i], addr[2i+1]). The digest is the sum
 * of the u16 results and the sum of result * (i & 0xffff), over nthreads host threads; packets are
 * regenerated on the fly, never materialised. */
#include <pthread.h>

static uint64_t inet_splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static void inet_splitmix_bytes(uint8_t *buf, size_t n, uint64_t seed, uint64_t pos0)
{
    size_t i = 0;
    for (; i < n && ((pos0 + i) & 7); i++)
        buf[i] = (uint8_t)(inet_splitmix64(seed + ((pos0 + i) >> 3)) >> (8 * ((pos0 + i) & 7)));
    for (; i + 8 <= n; i += 8) {   /* whole words (little-endian host) */
        const uint64_t w = inet_splitmix64(seed + ((pos0 + i) >> 3));
        memcpy(buf + i, &w, 8);
    }
    for (; i < n; i++)
        buf[i] = (uint8_t)(inet_splitmix64(seed + ((pos0 + i) >> 3)) >> (8 * ((pos0 + i) & 7)));
}

struct inet_digest_job {
    int mode;
    uint64_t seed, stride, i0, i1;
    const uint64_t *off;
    const uint32_t *len;
    const uint32_t *addr;
    uint32_t flen;
    uint64_t sum, wsum;
};

static void *inet_digest_worker(void *arg)
{
    struct inet_digest_job *j = (struct inet_digest_job *) arg;
    static __thread uint8_t buf[1 << 16];
    uint64_t sum = 0, wsum = 0;
    for (uint64_t i = j->i0; i < j->i1; i++) {
        const uint64_t o = j->off ? j->off[i] : i * j->stride;
        const uint32_t L = j->len ? j->len[i] : j->flen;
        if (L > sizeof buf)
            return NULL;   /* not for jumbo packets: sum stays short, the test fails loudly */
        inet_splitmix_bytes(buf, L, j->seed, o);
        uint16_t c;
        if (j->mode == 1)
            c = oracle_tcp_checksum(j->addr[2 * i], j->addr[2 * i + 1], buf, L);
        else if (j->mode == 2)
            c = oracle_udp_checksum(buf, L, j->addr[2 * i], j->addr[2 * i + 1]);
        else
            c = oracle_ip_checksum(buf, L);
        sum += c;
        wsum += (uint64_t) c * (i & 0xffffu);
    }
    j->sum = sum;
    j->wsum = wsum;
    return NULL;
}

void oracle_inet_splitmix_digest(int mode, uint64_t seed, const uint64_t *off, const uint32_t *len,
                                 uint64_t stride, uint32_t flen, const uint32_t *addr, uint64_t n, int nthreads,
                                 uint64_t *sum_out, uint64_t *wsum_out)
{
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    pthread_t th[256];
    struct inet_digest_job jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (struct inet_digest_job){mode, seed, stride, n * (uint64_t) t / (uint64_t) nthreads,
                                           n * (uint64_t)(t + 1) / (uint64_t) nthreads, off, len, addr, flen, 0, 0};
        pthread_create(&th[t], NULL, inet_digest_worker, &jobs[t]);
    }
    uint64_t sum = 0, wsum = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        sum += jobs[t].sum;
        wsum += jobs[t].wsum;
    }
    *sum_out = sum;
    *wsum_out = wsum;
}
