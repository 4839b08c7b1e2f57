// fcs_host_crc.hpp — the drop-in's last resort: CRC-32 on the host CPU.
//
// the reference ether_fcs (src/ether_fcs.c:4-19) cannot fail and has no
// error channel, so when the GPU path has failed twice (first attempt and the retry on a fresh
// lane), or the buffer is too large for the kernels' 32-bit frame lengths (>= 4 GiB), the drop-in
// returns this instead of aborting. Nothing else in the library calls it: every batch and device
// entry point stays GPU-only and fails with -errno. Each use is counted
// (fcs_engine_host_fallbacks) and announced once on stderr, and the GPU test suite asserts the
// count stays 0 (tests/test_gpu_dropin_recovery.py).
#pragma once
#include <cstddef>
#include <cstdint>

namespace fcs {

// ether_fcs(data, bsize) of the reference: CRC-32/ISO-HDLC, 0 for bsize == 0.
uint32_t host_crc32(const void *data, size_t bsize);

}  // namespace fcs
