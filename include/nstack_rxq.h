/*
 * nstack_rxq.h — batched RX call site for nstack's ether_receive, with FCS verification
 * (the call-site half of the RX row; the kernels are ether_fcs_verify_*).
 *
 * Reference: ether_receive(handle, hdr, buf, bsize), /root/reference/src/linux/ether.c:180-212,
 * reads one frame per call with recvfrom (:194-195), returns 0 when the socket has nothing
 * (EAGAIN / EWOULDBLOCK / EINPROGRESS, :196-198), skips frames whose source MAC is the
 * interface's own (:202), copies dst/src and the host-order ethertype into *hdr (:204-206) and
 * min(len - 14, bsize) payload bytes into buf (:208-209), and returns len - 14 (:211). It checks
 * no FCS: nstack's AF_PACKET socket normally receives frames without one.
 *
 * fcs_rxq_receive() keeps that per-call contract, but refills from the socket with one
 * recvmmsg (MSG_WAITFORONE: block as the socket is configured for the first frame, then take
 * whatever else is queued, up to max_batch) and hands the batch out one frame per call.
 * With FCS_RXQ_TRAILER (a link that delivers the 4-byte FCS, e.g. rx-fcs on) every batch is
 * verified (CRC residue) before any of its frames is handed out: on the GPU in one call
 * (pipelined with the next recvmmsg), or, below the GPU minimum (fcs_rxq_set_host_max), by the host
 * CRC on the receiving thread; frames that fail are dropped and counted, and the trailer is
 * stripped from the rest.
 * Deviations, both for frames the reference mishandles: a frame shorter than the header (plus
 * trailer) is dropped and counted (the reference's min() on a negative length is undefined), and a
 * frame longer than 1518 bytes (1514 + trailer) is dropped and counted (the reference truncates it
 * to its 1514-byte buffer). Errors: -errno from the socket (the reference returns -1 with errno
 * set). ether_receive never fails or drops a frame for FCS reasons, so when the GPU check of a
 * batch fails (HIP error, timeout, no GPU) the library's host CRC checks that batch instead
 * (SURVEY.md §8b): the frames come out exactly as they would have. Such batches are counted
 * (fcs_rxq_fallbacks, fcs_engine_host_batches) and the first is reported on stderr.
 * One consumer thread per queue (nstack's ingress thread); calls are serialised internally.
 */
#ifndef NSTACK_RXQ_H
#define NSTACK_RXQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fcs_rxq fcs_rxq_t;

/* struct ether_hdr of the reference (src/nstack_ether.h:54-58), packed like it, so a caller's
 * struct ether_hdr * converts without an alignment change: h_proto in host order on return. */
struct fcs_ether_hdr {
    uint8_t h_dst[6];
    uint8_t h_src[6];
    uint16_t h_proto;
} __attribute__((packed));

#define FCS_RXQ_TRAILER 1u   /* frames carry their 4-byte FCS: verify on the GPU, strip it */

/* fd: the receiving socket (AF_PACKET in nstack; any datagram socket works); own_mac: the
 * interface MAC whose echoes are skipped (eth->el_mac); max_batch: frames per recvmmsg (1..4096). */
fcs_rxq_t *fcs_rxq_create(int fd, const uint8_t own_mac[6], uint32_t max_batch, uint32_t flags);
/* ether_receive semantics: payload length (may exceed bsize; min(len, bsize) bytes are copied),
 * 0 when nothing is queued on a non-blocking / timed-out socket, or -errno (socket or engine). */
int fcs_rxq_receive(fcs_rxq_t *q, struct fcs_ether_hdr *hdr, uint8_t *buf, size_t bsize);
/* Counters since creation: frames received from the socket, frames that failed the FCS check,
 * own-MAC echoes skipped, runt or oversize frames dropped, recvmmsg batches. Any pointer may be NULL. */
void fcs_rxq_stats(const fcs_rxq_t *q, uint64_t *frames, uint64_t *bad_fcs, uint64_t *echoes,
                   uint64_t *dropped, uint64_t *batches);
/* Batches (and their frames) the host CRC checked because the GPU check failed. 0 on a healthy
 * GPU. Any pointer may be NULL. */
void fcs_rxq_fallbacks(const fcs_rxq_t *q, uint64_t *host_batches, uint64_t *host_frames);
/* GPU minimum: a received batch whose frames total at most `bytes` is checked by the library's host
 * CRC (fcs_host_crc32) on the receiving thread, where recvmmsg has just put the frames (cache-hot);
 * larger batches go to the GPU (pipelined with the next recvmmsg). Default 256 KiB, from the scan of
 * tools/rxq_host_max_scan.sh; NSTACK_RXQ_HOST_MAX_BYTES overrides it per process; 0 sends every batch to
 * the GPU. Returns the previous value (0 for NULL). */
uint64_t fcs_rxq_set_host_max(fcs_rxq_t *q, uint64_t bytes);
/* Batches (and frames) the host CRC checked by design (at or below the GPU minimum; failures are
 * fcs_rxq_fallbacks), and batches the GPU checked. Any pointer may be NULL. */
void fcs_rxq_small_batches(const fcs_rxq_t *q, uint64_t *small_batches, uint64_t *small_frames,
                           uint64_t *gpu_batches);
void fcs_rxq_destroy(fcs_rxq_t *q);

#ifdef __cplusplus
}
#endif
#endif /* NSTACK_RXQ_H */
