/*
 * nstack_inet.h — C ABI of the batched Internet-checksum kernels.
 *
 * An OPT-IN companion of the FCS engine in the same library (libnstack_fcs.so). nstack's
 * IP/TCP/UDP sources stay untouched (BASELINE.json north star); a caller that batches packets
 * can compute their checksums on the GPU through these entry points instead of the per-packet
 * loops. Every result is bit-identical to the reference function named by its mode:
 *
 *   INET_CSUM_IP   out[i] == ip_checksum(pkt, len)            /root/reference/src/ip.c:39-62
 *                  (declared src/nstack_ip.h:132; called by ip_hton src/ip.c:80 and the ICMP
 *                  replies src/icmp.c:42,74)
 *   INET_CSUM_TCP  out[i] == tcp_checksum(&src, &dst, pkt, len) /root/reference/src/tcp.c:167-213
 *                  (static; called by tcp_hton src/tcp.c:299). addr[2i] / addr[2i+1] are the
 *                  host-order source / destination IPv4 addresses (nstack_sockaddr.inet4_addr).
 *   INET_CSUM_UDP  out[i] == udp_checksum(pkt, len, src, dst)   /root/reference/src/udp.c:136-174
 *                  (static; called by nstack_udp_send src/udp.c:194). addr[2i] / addr[2i+1] are
 *                  the raw in_addr_t values that call passes.
 *
 * The value is the host-order uint16 the reference returns; stored with memcpy (as the
 * reference's callers do) its bytes are the on-wire checksum. A header or segment whose checksum
 * field already holds its checksum yields 0 (the receive-side checks src/ip.c:151 and
 * src/tcp.c:510, disabled in the reference). Lengths are the reference's size_t lengths; the
 * pseudo-header length field is htons(len), i.e. len mod 65536, as in the reference.
 *
 * There is no CPU path: without a usable gfx950 GPU the batch entry points return -ENODEV and the
 * single-packet forms abort with the reason on stderr (the reference functions have no error
 * channel). Errors: 0 or -errno (-EINVAL bad arguments, -ENODEV, -ENOMEM, -EIO); text in
 * fcs_last_error(). Thread-safe. Device forms run on the calling thread's current device and
 * are asynchronous on `stream` (a hipStream_t or NULL).
 */
#ifndef NSTACK_INET_H
#define NSTACK_INET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INET_CSUM_IP 0
#define INET_CSUM_TCP 1
#define INET_CSUM_UDP 2

/* ---- device-resident batches ---- */
/* Packet i = arena[off[i] .. off[i] + len[i]), inside [arena, arena + arena_bytes); off, len,
 * addr (2n u32; NULL for INET_CSUM_IP) and out are device arrays. */
int inet_csum_batch_dev(int mode, const void *arena, uint64_t arena_bytes, const uint64_t *off,
                        const uint32_t *len, const uint32_t *addr, uint16_t *out, uint64_t n,
                        void *stream);
/* Packet i = base[i*stride .. i*stride + len). stride >= len when n > 1. */
int inet_csum_fixed_dev(int mode, const void *base, uint64_t stride, uint32_t len, uint64_t n,
                        const uint32_t *addr, uint16_t *out, void *stream);

/* ---- host batches (host memory in and out; chunked H2D -> kernel -> D2H on the engine's
 *      first GPU; synchronous) ---- */
int inet_csum_batch_host(int mode, const void *arena, uint64_t arena_bytes, const uint64_t *off,
                         const uint32_t *len, const uint32_t *addr, uint16_t *out, uint64_t n);

/* Tuning: batches of more than `packets` packets use the flat kernel (packets dealt to lanes by
 * size, for throughput), smaller ones one 16-lane group per packet (latency); batches above the
 * DMA threshold (inet_csum_set_dma_threshold) take the LDS-DMA kernels instead.
 * Results are identical either way. Default 16384. Returns the previous value. */
uint64_t inet_csum_set_flat_threshold(uint64_t packets);

/* Tuning: batches of more than `packets` packets stream through LDS by DMA: fixed strides
 * (inet_csum_fixed_dev) four packets per wave item when the packets fill at least half their
 * stride (64..1532 B, stride <= 2048); variable batches in windows of 64 packets, each window whose
 * packets are packed and at least 16 B long as one span (the others by the flat kernel's method).
 * Results are identical either way. Default 16384. Returns the previous value. */
uint64_t inet_csum_set_dma_threshold(uint64_t packets);

/* ---- single packet, same arguments and result as the reference functions ---- */
uint16_t inet_ip_checksum(const void *dp, size_t bsize);                          /* ip.c:39  */
uint16_t inet_tcp_checksum(uint32_t src, uint32_t dst, const void *dp, size_t bsize); /* tcp.c:167 */
uint16_t inet_udp_checksum(const void *dp, size_t len, uint32_t src, uint32_t dst); /* udp.c:136 */

#ifdef __cplusplus
}
#endif

#endif /* NSTACK_INET_H */
