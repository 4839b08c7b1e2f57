// fcs_device.hpp — device lookup shared by the library's translation units (not exported).
#pragma once
#include <stdint.h>

#include <functional>

namespace fcs {
// The calling thread's current HIP device, checked to be a gfx950 (lazily initialised engine
// state). Returns 0 or -errno (with fcs_last_error() set).
__attribute__((visibility("hidden"))) int current_device(int *dev, int *cus);
// The first device of the engine's device set (fcs_engine_init), for the host entry points.
__attribute__((visibility("hidden"))) int engine_device0(int *dev, int *cus);
// memcpy into pinned staging, split over a few threads for large spans (host pipelines).
__attribute__((visibility("hidden"))) void staging_copy(uint8_t *dst, const uint8_t *src, uint64_t bytes);
// Asynchronous RX residue check over frames in fcs_host_alloc memory (the small-batch kernel reading
// its frame list from mapped memory): arena, off, len and ok must all lie in fcs_host_alloc ranges,
// every len <= 1536; ok[i] = 1 / 0. Launches and returns a ticket, or -errno (nothing launched).
// Results are in place once mapped_wait(ticket) returned 0; tickets complete in the order they were
// issued. A failed wait leaves the kernel in flight: it may still write ok[] (the caller sets the
// array aside); the engine retires its own stream and words, and waits for tickets issued before
// that fail with -EIO.
__attribute__((visibility("hidden"))) int mapped_submit(uint8_t *arena, uint64_t arena_bytes, const uint64_t *off,
                                                        const uint32_t *len, uint8_t *ok, uint64_t n,
                                                        uint64_t *ticket);
__attribute__((visibility("hidden"))) int mapped_wait(uint64_t ticket);
// A host batch call or TX/RX queue batch whose GPU step failed was answered by the host CRC
// (fcs_host_crc.cpp): counted in fcs_engine_host_batches(), the first one reported on stderr with
// the site and reason.
__attribute__((visibility("hidden"))) void host_batch_answered(const char *site, const char *why);
// True when the calling thread's last ether_fcs_*_host call was answered by the host CRC (the
// queues count their own batches with it).
__attribute__((visibility("hidden"))) bool last_call_host_answered();
// Runs launch(ctr) with a zeroed work counter of device `dev` (the Dispenser's, dispenser.hpp)
// leased for that launch on stream `stream` (a hipStream_t; zeroed on it after the slot's previous
// kernel finished). Host-only headers include this file, so the stream travels as void *.
__attribute__((visibility("hidden"))) int launch_with_counter(int dev, void *stream,
                                                              const std::function<int(unsigned long long *)> &launch);
}  // namespace fcs
