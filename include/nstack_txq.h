/*
 * nstack_txq.h — batched TX call site for nstack's ether_send.
 *
 * Reference: ether_send(handle, dst, proto, buf, bsize), /root/reference/src/linux/ether.c:214-272,
 * builds one frame in a stack VLA, computes its FCS with ether_fcs (:262), stores it
 * little-endian after the covered bytes (:263) and calls sendto once per frame (:265). Its
 * callers (ether_output_reply, src/ether.c:39-53; ip_send, arp) run on the main, ingress,
 * egress and TCP-timer threads concurrently.
 *
 * fcs_txq_send() keeps that contract per call — same frame bytes, same return value (bytes sent
 * or -errno), same -EMSGSIZE rule — but frames from all producer threads are assembled into one
 * pinned batch arena, their FCSs are computed together on the GPU (ether_fcs_tx_batch_host; where
 * the GPU does not pay, on the host: see fcs_txq_set_host_max), and the batch leaves through one
 * sink call (sendmmsg for the provided sinks). A batch is flushed when it
 * holds max_batch frames, or the flusher is idle and the batch's oldest frame has lingered
 * flush_usec microseconds (0: leave as soon as the flusher is free). The queue double-buffers:
 * producers fill batch k+1 while batch k is on the GPU/wire, so batches grow with the offered
 * load by themselves and a linger is only worth it for fire-and-forget senders.
 * fcs_txq_send() blocks until its own frame has been handed to the sink and returns that frame's
 * result. ether_send never fails for FCS reasons (it fails only on -EMSGSIZE, a bad handle or
 * sendto, :234-269), so if the GPU step fails (HIP error, timeout, no GPU) the batch's FCSs are
 * computed by the library's host CRC instead and the frames leave as usual: the
 * per-call results never depend on the GPU. Such batches are counted (fcs_txq_fallbacks,
 * fcs_engine_host_batches), the first is reported on stderr, and fcs_txq_last_error keeps the
 * reason. A failed step's pinned arena is set aside (a late kernel may still write into it); after
 * 16 such batches the queue stops calling the GPU and stays on the host CRC.
 */
#ifndef NSTACK_TXQ_H
#define NSTACK_TXQ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fcs_txq fcs_txq_t;

/* Transmit n finished frames (header + payload + pad + FCS; sizes[i] bytes at frames[i]).
 * Must store each frame's result in res[i]: bytes sent, or -errno (as sendto's result at
 * src/linux/ether.c:265-269). Must be thread-safe: the flusher thread calls it one batch at a time,
 * and synchronous senders call it from their own threads with a batch of one frame, concurrently
 * (see fcs_txq_set_sync_host), as nstack's threads call sendto concurrently. The provided sinks are. */
typedef void (*fcs_txq_sink_fn)(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res,
                                uint32_t n);

/* src_mac: the interface MAC ether_send copies into h_src (eth->el_mac, :258).
 * max_batch: frames per batch (1 .. 65536); flush_usec: linger of a non-full batch (see above). */
fcs_txq_t *fcs_txq_create(const uint8_t src_mac[6], uint32_t max_batch, uint32_t flush_usec,
                          fcs_txq_sink_fn sink, void *sink_ctx);
/* ether_send semantics: returns frame_size = 14 + max(bsize, 56) + 4 on success, -EMSGSIZE when
 * that exceeds 1518 (checked before anything is queued, :234-237), or the sink's / engine's
 * -errno. Thread-safe; returns once the frame has been handed to the sink (sent by the caller itself
 * or in its batch). */
int fcs_txq_send(fcs_txq_t *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize);
/* Fire-and-forget form: returns frame_size once the frame is queued (or -EMSGSIZE / -EINVAL);
 * its send result only feeds the error counter of fcs_txq_stats. */
int fcs_txq_send_async(fcs_txq_t *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf,
                       size_t bsize);
/* Flush whatever is queued now and wait for it. Returns 0 or -errno (bad queue). */
int fcs_txq_flush(fcs_txq_t *q);
/* Flushes, stops the flusher thread and frees the queue. */
void fcs_txq_destroy(fcs_txq_t *q);
/* Counters since creation: frames handed to the sink, batches, and frames whose result was not
 * frame_size (sink errors). Any pointer may be NULL. */
void fcs_txq_stats(const fcs_txq_t *q, uint64_t *frames, uint64_t *batches, uint64_t *errors);
/* Flusher time since creation, in ns, summed over batches: waiting for producers to finish
 * assembling, the GPU step (ether_fcs_tx_host), the sink, the whole per-batch busy time (their
 * sum plus bookkeeping), and pickup (a batch's first frame queued -> the flusher closing it). */
void fcs_txq_timing(const fcs_txq_t *q, uint64_t *ns_ready, uint64_t *ns_gpu, uint64_t *ns_sink,
                    uint64_t *ns_busy, uint64_t *ns_pickup);
/* Text of the most recent failed GPU step (fcs_last_error() of the flusher thread when its
 * ether_fcs_tx_batch_host call failed); "" when no batch has failed. Valid until the next call. */
const char *fcs_txq_last_error(const fcs_txq_t *q);
/* Batches (and their frames) whose FCSs the host CRC computed because the GPU step failed; the
 * frames were sent all the same. 0 on a healthy GPU. Any pointer may be NULL. */
void fcs_txq_fallbacks(const fcs_txq_t *q, uint64_t *host_batches, uint64_t *host_frames);
/* Where the GPU does not pay, the library's host CRC (fcs_host_crc32) computes the FCS, by design:
 * a GPU step costs a launch and a completion round trip (9-12 us on MI355X) whatever it holds, a
 * hand-off between threads 1-2 us, and the host CRC about 0.03 us per 1518-B frame.
 * - fcs_txq_send (synchronous): a caller with none of its own frames queued sends its frame itself
 *   (ether_send's body with the host CRC; the sink gets a batch of one on the caller's thread); a
 *   caller with fire-and-forget frames queued joins their batch (order kept) and computes its own
 *   frame's FCS there. fcs_txq_set_sync_host(q, 0) turns this off: synchronous frames then join the
 *   batch and take its GPU step. Returns the previous setting (1 = on, the default) or -EINVAL.
 * - fcs_txq_send_async (fire-and-forget): the frames of one batch take one GPU step when their
 *   FCS-covered bytes total more than `bytes`, the GPU minimum; at or below it the flusher computes
 *   them. The default (16 KiB) comes from the in-queue scan of tools/txq_vs_reference.sh; it can be
 *   overridden per process by NSTACK_TXQ_HOST_MAX_BYTES; 0 sends every batch to the GPU.
 *   fcs_txq_set_host_max returns the previous value (0 for a NULL queue). */
uint64_t fcs_txq_set_host_max(fcs_txq_t *q, uint64_t bytes);
int fcs_txq_set_sync_host(fcs_txq_t *q, int on);
/* Batches that took no GPU step and frames whose FCS the host CRC computed, both by design (callers'
 * own frames and batches at or below the GPU minimum; not failures: those are fcs_txq_fallbacks), and
 * batches whose FCSs a GPU step computed. Any pointer may be NULL. */
void fcs_txq_small_batches(const fcs_txq_t *q, uint64_t *small_batches, uint64_t *small_frames,
                           uint64_t *gpu_batches);

/* ---- provided sinks ---- */
/* ctx = pointer to an int file descriptor of a CONNECTED socket (e.g. a socketpair or a
 * connected AF_PACKET/UDP socket): one sendmmsg per batch (send for a batch of one), no
 * per-message address. */
void fcs_txq_sink_fd(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res, uint32_t n);
/* AF_PACKET raw socket, as ether_send uses it (:241-253): ctx = struct fcs_txq_packet_ctx*.
 * Each frame's sockaddr_ll takes sll_protocol and sll_addr from the frame's own header; one
 * sendmmsg per batch, sendto for a batch of one (exactly ether_send's call). */
struct fcs_txq_packet_ctx {
    int fd;
    int ifindex;
};
void fcs_txq_sink_packet(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif /* NSTACK_TXQ_H */
