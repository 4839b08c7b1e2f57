// inet_launch.hpp — host-side launcher of the Internet-checksum kernel (inet_kernel.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace inet {

// Modes = the reference function whose return value out[i] reproduces (include/nstack_inet.h).
constexpr int kIp = 0;    // ip_checksum   src/ip.c:39-62
constexpr int kTcp = 1;   // tcp_checksum  src/tcp.c:167-213
constexpr int kUdp = 2;   // udp_checksum  src/udp.c:136-174

struct IParams {
    uint64_t base;          // fixed: packet 0 start; var: arena start
    uint64_t stride;        // fixed only
    const uint64_t *off;    // var only
    const uint32_t *len;    // var only
    const uint32_t *addr;   // tcp/udp: (src, dst) per packet
    uint16_t *out;
    uint64_t n;
    uint32_t flen;          // fixed: packet length
    unsigned long long *ctr;   // inet_dma_kernel: zeroed device work counter (fcs::launch_with_counter)
};

// Fixed-stride batches of more than dma_min packets whose four-packet items fit a 6 KiB slot take
// the LDS-DMA kernel; otherwise batches of more than flat_min packets take the flat chunk-stream
// kernel, smaller ones one 16-lane group per packet (every packet in flight at once).
hipError_t launch_inet(bool var, int mode, const IParams &p, int cus, uint64_t flat_min, uint64_t dma_min,
                       hipStream_t st);
// The kernel launch_inet takes: kStream (variable batches of more than dma_min packets: windows
// interleaved statically, like the flat kernel's; guided chunks measured 4 % slower there on IMIX,
// 17 % on 20-B headers), kShort (fixed packets of at most 64 B, more than flat_min), kDma (fixed
// strides of more than dma_min packets whose items fit a slot: inet_dma_kernel, the only one that
// needs p.ctr), kFlat (more than flat_min), kGroup (a 16-lane group per packet), kNone (n == 0).
enum class Route { kNone, kStream, kShort, kDma, kFlat, kGroup };
Route route_inet(bool var, const IParams &p, uint64_t flat_min, uint64_t dma_min);

}  // namespace inet
