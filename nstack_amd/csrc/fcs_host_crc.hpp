// fcs_host_crc.hpp — the library's host CRC-32: the last resort of the reference-contract call sites,
// and the TX queue's answer for batches below its GPU minimum (fcs_txq.cpp).
//
// the reference ether_fcs (src/ether_fcs.c:4-19) cannot fail and has no
// error channel, and ether_send / ether_receive (src/linux/ether.c:180-272) never fail for FCS
// reasons. So the drop-in returns this when the GPU path has failed twice (first attempt and the
// retry on a fresh lane) or the buffer is too large for the kernels' 32-bit frame lengths (>= 4 GiB);
// the host batch forms (ether_fcs_*_host) compute or check a batch with it when their GPU step fails
// with a runtime error; and the TX/RX queues use it when no GPU is usable at all. The device forms
// stay GPU-only and fail with -errno. Each use is counted (fcs_engine_host_fallbacks,
// fcs_engine_host_batches) and announced once on stderr, and the GPU test suite asserts both counts
// stay 0 (tests/test_gpu_zz_no_host_fallback.py). It is the product's own code, not the test oracle.
#pragma once
#include <cstddef>
#include <cstdint>

namespace fcs {

// ether_fcs(data, bsize) of the reference: CRC-32/ISO-HDLC, 0 for bsize == 0. Carry-less folding
// when the CPU has PCLMULQDQ, else the tables.
uint32_t host_crc32(const void *data, size_t bsize);
// The same CRC through the slice-by-16 tables only (the form without PCLMULQDQ; tests compare both).
uint32_t host_crc32_tables(const void *data, size_t bsize);

}  // namespace fcs
