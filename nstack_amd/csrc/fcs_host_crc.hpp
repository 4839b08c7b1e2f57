// fcs_host_crc.hpp — the last resort of the reference-contract call sites: CRC-32 on the host CPU.
//
// the reference ether_fcs (src/ether_fcs.c:4-19) cannot fail and has no
// error channel, and ether_send / ether_receive (src/linux/ether.c:180-272) never fail for FCS
// reasons. So when the GPU path has failed twice (first attempt and the retry on a fresh lane), or
// the buffer is too large for the kernels' 32-bit frame lengths (>= 4 GiB), the drop-in returns
// this instead of aborting; and when the GPU step of a TX or RX queue batch fails, the queue
// computes or checks that batch's FCSs with it instead of failing or dropping the frames. The
// batch and device entry points stay GPU-only and fail with -errno. Each use is counted
// (fcs_engine_host_fallbacks, fcs_engine_host_batches) and announced once on stderr, and the GPU
// test suite asserts both counts stay 0 (tests/test_gpu_zz_no_host_fallback.py).
#pragma once
#include <cstddef>
#include <cstdint>

namespace fcs {

// ether_fcs(data, bsize) of the reference: CRC-32/ISO-HDLC, 0 for bsize == 0.
uint32_t host_crc32(const void *data, size_t bsize);

}  // namespace fcs
