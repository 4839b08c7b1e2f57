/*
 * nstack_fcs.h — C ABI of the MI355X Ethernet FCS (IEEE 802.3 CRC-32) engine.
 *
 * Drop-in boundary for nstack's FCS path. Every entry point is plain C (no HIP/torch types):
 * pointers, sizes, and an opaque `void *stream` (a hipStream_t, or NULL for the default stream).
 *
 * Reference interfaces replaced / served:
 *   ether_fcs()                 replaces uint32_t ether_fcs(const void *, size_t)
 *                               declared /root/reference/src/nstack_ether.h:80,
 *                               defined   /root/reference/src/ether_fcs.c:4-19.
 *                               Link libnstack_fcs.so in place of ether_fcs.o
 *                               (/root/reference/Makefile:13) — no caller changes.
 *   ether_fcs_batch_host()      the batched form of the per-frame call in ether_send()
 *   ether_fcs_fixed_host()      (/root/reference/src/linux/ether.c:262); see INTEGRATION.md.
 *   ether_fcs_tx_host()         TX mode of the same call site: computes the FCS over the first
 *                               len bytes of each frame and stores it little-endian right after
 *                               them, exactly as src/linux/ether.c:262-263 does per frame.
 *   ether_fcs_tx_batch_host()   the same over arena + offsets (the TX queue's batches).
 *   ether_fcs_*_dev()           device-resident forms (frames already in HBM).
 *
 * Semantics (all entry points): out[i] == ether_fcs(frame_i, len_i) of the reference, i.e.
 * CRC-32/ISO-HDLC (reflected poly 0xEDB88320, init/final complement), bit-exact; len 0 -> 0.
 *
 * Errors (the reference's ether_fcs cannot fail). Every entry point returns 0 on
 * success or a negative errno; fcs_last_error() has the text.
 *   -EINVAL   bad arguments: nothing has been written. Never answered by the host CRC.
 *   -ENODEV   no usable gfx950 GPU or HIP code object at all: the batch and device forms fail
 *             loudly then (they never turn into a CPU library). The drop-in ether_fcs is the
 *             exception below.
 *   device forms (*_dev): any other HIP error is returned (-EIO, -ENOMEM, ...): the frames are in
 *             device memory, so there is no host answer to give.
 *   host forms (ether_fcs_batch_host, _fixed_host, _tx_host, _tx_batch_host, _verify_host): any
 *             other failure of the GPU step (a HIP error, a lost completion, the 10 s timeout, an
 *             allocation failure) is answered by the library's own host CRC (fcs_host_crc32,
 *             fcs_host_crc.cpp; not a test oracle), so the results are the reference's and the call
 *             returns 0 (verify: the bad count). Each such call is counted in
 *             fcs_engine_host_batches(), the first is reported on stderr, and fcs_last_error() says
 *             "<form> answered by the host CRC after: <the GPU error>". A failed GPU step never leaves
 *             a kernel that can write into the caller's memory: results travel through the library's
 *             own staging and mapped arrays, which are set aside (never reused or freed before
 *             fcs_engine_fini) when a kernel may still be in flight. After 16 such set-asides the
 *             host forms stop calling the GPU and answer from the host CRC (counted) until
 *             fcs_engine_fini. fcs_host_free waits up to 10 s for set-aside kernels before it frees
 *             pinned memory, and keeps the memory if one is still running.
 *   ether_fcs (drop-in): a failed attempt (HIP error, lost completion, timeout) quarantines that
 *             lane's stream and result word and is retried once on a fresh lane; if the retry fails
 *             too, or there is no GPU, or bsize >= 4 GiB (the kernels take 32-bit lengths), the call
 *             is answered by the same host CRC instead of aborting. Counted in
 *             fcs_engine_host_fallbacks, first reported on stderr; fcs_engine_stats counts calls,
 *             retries and recoveries.
 * The TX/RX call-site queues (nstack_txq.h, nstack_rxq.h) go through the host forms, so they keep
 * ether_send's / ether_receive's contract: never failed or dropped for FCS reasons.
 *
 * Threading: every entry point is thread-safe and may be called concurrently (the reference
 * calls ether_fcs from the main, ingress, egress and TCP-timer threads: SURVEY.md §8b).
 * Device entry points run on the calling thread's current HIP device; the caller owns all
 * buffers until the call returns (host forms, synchronous) or until the stream reaches the
 * point after the call (device forms, asynchronous).
 */
#ifndef NSTACK_FCS_H
#define NSTACK_FCS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- drop-in single frame (src/ether_fcs.c:4, src/nstack_ether.h:80) ---- */
uint32_t ether_fcs(const void *data, size_t bsize);

/* ---- engine lifetime (optional: every entry point initialises lazily) ---- */
/* Use the first ndev visible GPUs (ndev <= 0: all). Returns the device count or -errno. */
int fcs_engine_init(int ndev);
void fcs_engine_fini(void);
int fcs_engine_device_count(void);
const char *fcs_last_error(void);
/* Engine/kernel description string (kernel geometry and table layout). */
const char *fcs_engine_version(void);
/* Tuning: variable-length batches of at most `frames` frames use the latency-optimised kernel
 * (one quarter-wave per frame), larger ones the throughput-optimised windowed kernel. Results are
 * identical either way. Default 16384. Returns the previous value. */
uint64_t fcs_engine_set_var_threshold(uint64_t frames);
/* Drop-in health: ether_fcs calls, first attempts that failed and were retried, retries that
 * succeeded, and lanes (stream + result word) dropped after a failure. Any pointer may be NULL. */
void fcs_engine_stats(uint64_t *dropin_calls, uint64_t *dropin_retries, uint64_t *dropin_recovered,
                      uint64_t *lane_resets);
/* Drop-in calls answered by the host CRC because the GPU path failed twice or bsize >= 4 GiB
 * (0 on a healthy GPU: the GPU test suite asserts it). */
uint64_t fcs_engine_host_fallbacks(void);
/* Host batch calls (ether_fcs_*_host, including the TX/RX call-site queues' batches, nstack_txq.h,
 * nstack_rxq.h) whose GPU step failed and whose results were therefore computed or checked by the
 * same host CRC, so that their results, and ether_send's and ether_receive's per-call results,
 * never depend on the GPU (0 on a healthy GPU: the GPU test suite asserts it). */
uint64_t fcs_engine_host_batches(void);
/* Host batch paths: calls that were split over more than one engine device, and the shard jobs
 * those calls ran (one host thread and pipeline each). Any pointer may be NULL. */
void fcs_engine_host_stats(uint64_t *sharded_calls, uint64_t *shard_jobs);
/* Shard planner of the host batch paths (and of bench.py's ranks): cut[0..parts] such that part g
 * is frames [cut[g], cut[g+1]). len == NULL: equal frame counts (cut[g] = n g / parts); otherwise
 * byte-balanced contiguous ranges (cut[g] = first index whose length prefix reaches g/parts of the
 * total). Pure host arithmetic, no GPU needed. Returns 0 or -EINVAL. */
int fcs_shard_plan(const uint32_t *len, uint64_t n, uint32_t parts, uint64_t *cut);

/* ---- device-resident batches (pointers in HBM of the current device) ---- */
/* Variable-length frames: frame i = arena[off[i] .. off[i]+len[i]), all inside
 * [arena, arena + arena_bytes). off/len/out are device arrays of n elements. */
int ether_fcs_batch_dev(const void *arena, uint64_t arena_bytes, const uint64_t *off,
                        const uint32_t *len, uint32_t *out, uint64_t n, void *stream);
/* Fixed-length frames: frame i = base[i*stride .. i*stride+len). stride >= len. */
int ether_fcs_fixed_dev(const void *base, uint64_t stride, uint32_t len, uint64_t n,
                        uint32_t *out, void *stream);

/* ---- host batches (host memory in and out; sharded over the engine's GPUs,
 *      chunked H2D -> kernel -> D2H pipeline per GPU; synchronous) ----
 * The arena forms check every frame (and, in TX mode, its FCS bytes) against the arena before
 * any work: on -EINVAL, which names the first bad frame, nothing has been written. */
int ether_fcs_batch_host(const void *arena, uint64_t arena_bytes, const uint64_t *off,
                         const uint32_t *len, uint32_t *out, uint64_t n);
int ether_fcs_fixed_host(const void *base, uint64_t stride, uint32_t len, uint64_t n,
                         uint32_t *out);
/* TX mode (src/linux/ether.c:262-263): frame i occupies base[i*stride ..]; the FCS over its
 * first len[i] bytes is written little-endian at base[i*stride + len[i] .. +4). Requires
 * len[i] + 4 <= stride. Frames are modified in place in host memory. */
int ether_fcs_tx_host(void *base, uint64_t stride, const uint32_t *len, uint64_t n);
/* TX mode over the packed-arena layout: frame i is arena[off[i] .. +len[i]) and
 * its FCS goes to arena[off[i] + len[i] .. +4), which must lie inside [arena, arena +
 * arena_bytes). Frames must not overlap each other's FCS bytes. Batches of up to 64 MiB in
 * fcs_host_alloc memory are read and answered in place (no staging copies). */
int ether_fcs_tx_batch_host(void *arena, uint64_t arena_bytes, const uint64_t *off,
                            const uint32_t *len, uint64_t n);

/* ---- RX verification (new behaviour: the reference's ether_receive,
 *      src/linux/ether.c:180-212, checks no FCS) ----
 * Frames here INCLUDE their 4-byte FCS trailer (len[i] = covered bytes + 4). A frame checks iff
 * ether_fcs(frame, len) == 0x2144DF1C, the CRC-32 residue, which holds exactly when the trailer
 * is the little-endian FCS of the bytes before it, as ether_send (src/linux/ether.c:262-263)
 * writes it. ok[i] = 1 / 0; frames shorter than 4 bytes never check.
 * Device forms: ok[] and *bad (u64) are device memory; *bad is zeroed on the stream, then set to
 * the number of failing frames. Host form: returns that number (>= 0) or -errno. */
int ether_fcs_verify_dev(const void *arena, uint64_t arena_bytes, const uint64_t *off,
                         const uint32_t *len, uint8_t *ok, uint64_t *bad, uint64_t n, void *stream);
int ether_fcs_verify_fixed_dev(const void *base, uint64_t stride, uint32_t len, uint64_t n,
                               uint8_t *ok, uint64_t *bad, void *stream);
int64_t ether_fcs_verify_host(const void *arena, uint64_t arena_bytes, const uint64_t *off,
                              const uint32_t *len, uint8_t *ok, uint64_t n);

/* ---- the library's own host CRC (never the GPU) ----
 * ether_fcs(data, bsize) computed on the calling CPU: carry-less folding, four 128-bit lanes wide
 * with AVX-512 VPCLMULQDQ or one lane with PCLMULQDQ (chosen at run time; ~32 ns per 1518-B frame and
 * ~79 GB/s on 64 KiB on one EPYC 9575F core, profiles/r06_host_crc_forms.jsonl), or slice-by-16
 * tables, all derived from the polynomial at run time (fcs_host_crc.cpp). It is what the failure paths above answer with and what the TX queue
 * computes batches below its GPU minimum with (nstack_txq.h, fcs_txq_set_host_max). Exported so
 * callers and tests can see the exact function those paths use; no GPU form falls back to it. */
uint32_t fcs_host_crc32(const void *data, size_t bsize);

/* ---- pinned host memory for zero-copy-staging callers (optional) ----
 * Pinned, device-mapped, portable host memory. TX and verify batches of up to 64 MiB in it are
 * read by the kernel in place. Release it with fcs_host_free only (the engine keeps the range's
 * device address until then). */
void *fcs_host_alloc(uint64_t bytes);
void fcs_host_free(void *p);

/* ---- measurement helpers (used by bench.py; not part of the reference surface) ---- */
/* Fill [p, p+bytes) of device memory with the counter-based splitmix64 stream:
 * byte at stream position q = byte_offset + i is byte (q & 7) of splitmix64(seed + q/8). */
int fcs_fill_splitmix64_dev(void *p, uint64_t bytes, uint64_t seed, uint64_t byte_offset,
                            void *stream);
/* Pure HBM read-stream kernel over [p, p+bytes): the measured read ceiling. */
int fcs_read_stream_dev(const void *p, uint64_t bytes, uint32_t *sink, void *stream);
/* The LDS-DMA read ceiling: the headline kernel's slot DMA (global_load_lds, nt), schedule and
 * window reads over [p, p+bytes) viewed as 1518-B frames, without the CRC work. */
int fcs_dma_stream_dev(const void *p, uint64_t bytes, uint32_t *sink, void *stream);
/* The arena-stream kernel's own load ceiling (fcs_stream_kernel<true>): a windowed variable-length
 * batch's units, unit check, 4 KiB items, slot DMA and schedule exactly as ether_fcs_batch_dev runs
 * them, without the marks, chain, chunk contributions or closes; sink receives nothing (a store no
 * realistic input triggers). Measurement only (bench.py configs.imix_128M.stream_load_gbs). */
int fcs_stream_load_dev(const void *arena, uint64_t arena_bytes, const uint64_t *off, const uint32_t *len,
                        uint64_t n, uint32_t *sink, void *stream);
/* Average device time (ms) per launch of the last `reps` timed FCS launches measured with
 * HIP events on the launch stream: fcs_timed_fixed_dev() launches ether_fcs_fixed_dev
 * `reps` times back to back, bracketed by events recorded on `stream`. */
int fcs_timed_fixed_dev(const void *base, uint64_t stride, uint32_t len, uint64_t n,
                        uint32_t *out, void *stream, int reps, float *ms_per_launch);

/* Test introspection: the number of units (fcs_debug_stream_unit_frames() frames each) the last
 * arena-stream launch (windowed variable-length batches) left to fcs_flat_kernel because their
 * frames are not packed or not 64..1536 B long; -1 before any. Synchronises
 * the device. */
int64_t fcs_debug_stream_listed(void);
uint32_t fcs_debug_stream_unit_frames(void);
/* Test introspection: the kernel a fixed-length batch (frames of len bytes every stride bytes from
 * base, n frames) would take, as ether_fcs_fixed_dev picks it (fcs::route_fixed, the one function
 * that decides it): "short:W", "flat", "wide4:WD", "wide8:WD", "wide16:WD", "segment", "lds-dma",
 * "tiny", "single" or "generic" (DESIGN.md §3.2). Host arithmetic only: no device call, base is not
 * read. Writes a NUL-terminated name into out (cap bytes); returns its length or -errno. */
int fcs_debug_fixed_route(uint64_t base, uint64_t stride, uint32_t len, uint64_t n, char *out, uint64_t cap);
/* Test introspection: the kernel the process's last fixed-length launch actually launched, recorded
 * by the launcher in the branch that launches it: "<name as above>/<workgroup threads>", or "none". */
int fcs_debug_last_fixed_launch(char *out, uint64_t cap);
/* Test introspection: device-wide synchronisations the engine has issued since load. The paths that
 * run after a failed call set a kernel aside (a retired stream that may never finish) issue none. */
uint64_t fcs_debug_device_syncs(void);
/* Test introspection: copy the constant tables the kernel stages into LDS (GF(2) operators of
 * the CRC, built on the host once; no frame data involved). Returns words written or -errno. */
int fcs_tables_blob(uint32_t *out, uint64_t words);

#ifdef __cplusplus
}
#endif
#endif /* NSTACK_FCS_H */
