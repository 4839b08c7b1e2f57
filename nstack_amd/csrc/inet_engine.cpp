// inet_engine.cpp — the C ABI of include/nstack_inet.h around inet_kernel.hip.
//
// Device forms validate and launch; the host form runs a double-buffered H2D -> kernel -> D2H
// pipeline of 128 MiB chunks on the engine's first GPU (packets of a chunk are copied as one span
// when they lie densely, gathered into the pinned staging buffer otherwise). The single-packet
// forms keep the reference functions' signatures (src/ip.c:39, src/tcp.c:167, src/udp.c:136) and,
// like them, have no error channel: on an engine failure they abort with the reason.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>

#include "../../include/nstack_fcs.h"
#include "../../include/nstack_inet.h"
#include "fcs_device.hpp"
#include "fcs_error.hpp"
#include "inet_launch.hpp"

namespace {

int hip_fail(hipError_t e, const char *what) {
    const int err = (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu ||
                     e == hipErrorInvalidDeviceFunction || e == hipErrorInvalidImage)
                        ? ENODEV
                        : (e == hipErrorOutOfMemory ? ENOMEM : EIO);
    return fcs::set_error(err, "%s: %s", what, hipGetErrorString(e));
}

#define HIPTRY(expr, what)                                 \
    do {                                                   \
        hipError_t e_ = (expr);                            \
        if (e_ != hipSuccess) return hip_fail(e_, what);   \
    } while (0)

std::atomic<uint64_t> g_flat_min{16384};   // see inet_csum_set_flat_threshold
std::atomic<uint64_t> g_dma_min{16384};    // see inet_csum_set_dma_threshold

// launch_inet with the work counter the LDS-DMA route takes (the same route_inet decision the
// launcher makes), leased from the FCS engine's ring of device `dev` for this launch.
int launch_counted(bool var, int mode, inet::IParams &p, int dev, int cus, hipStream_t st) {
    const uint64_t flat_min = g_flat_min.load(std::memory_order_relaxed), dma_min = g_dma_min.load(std::memory_order_relaxed);
    auto go = [&](unsigned long long *ctr) -> int {
        p.ctr = ctr;
        HIPTRY(inet::launch_inet(var, mode, p, cus, flat_min, dma_min, st), "launching the inet kernel");
        return 0;
    };
    if (inet::route_inet(var, p, flat_min, dma_min) == inet::Route::kDma)
        return fcs::launch_with_counter(dev, (void *)st, go);
    return go(nullptr);
}

int check_mode(int mode, const uint32_t *addr) {
    if (mode != INET_CSUM_IP && mode != INET_CSUM_TCP && mode != INET_CSUM_UDP)
        return fcs::set_error(EINVAL, "unknown checksum mode %d", mode);
    if (mode != INET_CSUM_IP && !addr) return fcs::set_error(EINVAL, "mode %d needs the address array", mode);
    return 0;
}

// ---- host pipeline ----
constexpr uint64_t kChunkBytes = 128ull << 20;
constexpr uint64_t kChunkPkts = 1ull << 20;
constexpr int kDepth = 2;

struct Slot {
    uint8_t *d_in = nullptr, *h_in = nullptr;
    uint64_t *d_off = nullptr, *h_off = nullptr;
    uint32_t *d_len = nullptr, *h_len = nullptr, *d_addr = nullptr, *h_addr = nullptr;
    uint16_t *d_out = nullptr, *h_out = nullptr;
    hipEvent_t done = nullptr;
    bool live = false;
    uint64_t i0 = 0, n = 0;
};

struct HostPipe {
    std::mutex mu;
    int dev = -1, cus = 0;
    hipStream_t stream = nullptr;
    Slot slot[kDepth];
};

std::mutex g_pipes_mu;
std::map<int, std::unique_ptr<HostPipe>> g_pipes;

int get_pipe(int dev, int cus, HostPipe **out) {
    std::lock_guard<std::mutex> lk(g_pipes_mu);
    auto &up = g_pipes[dev];
    if (!up) {
        auto hp = std::make_unique<HostPipe>();
        hp->dev = dev;
        hp->cus = cus;
        HIPTRY(hipSetDevice(dev), "hipSetDevice");
        HIPTRY(hipStreamCreateWithFlags(&hp->stream, hipStreamNonBlocking), "hipStreamCreate");
        for (Slot &s : hp->slot) {
            HIPTRY(hipMalloc(&s.d_in, kChunkBytes + 64), "hipMalloc(inet staging)");
            HIPTRY(hipHostMalloc(&s.h_in, kChunkBytes + 64, hipHostMallocDefault), "hipHostMalloc(inet staging)");
            HIPTRY(hipMalloc(&s.d_off, kChunkPkts * 8), "hipMalloc(off)");
            HIPTRY(hipHostMalloc(&s.h_off, kChunkPkts * 8, hipHostMallocDefault), "hipHostMalloc(off)");
            HIPTRY(hipMalloc(&s.d_len, kChunkPkts * 4), "hipMalloc(len)");
            HIPTRY(hipHostMalloc(&s.h_len, kChunkPkts * 4, hipHostMallocDefault), "hipHostMalloc(len)");
            HIPTRY(hipMalloc(&s.d_addr, kChunkPkts * 8), "hipMalloc(addr)");
            HIPTRY(hipHostMalloc(&s.h_addr, kChunkPkts * 8, hipHostMallocDefault), "hipHostMalloc(addr)");
            HIPTRY(hipMalloc(&s.d_out, kChunkPkts * 2), "hipMalloc(out)");
            HIPTRY(hipHostMalloc(&s.h_out, kChunkPkts * 2, hipHostMallocDefault), "hipHostMalloc(out)");
            HIPTRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming), "hipEventCreate");
        }
        up = std::move(hp);
    }
    *out = up.get();
    return 0;
}

int run_host(int mode, const uint8_t *arena, const uint64_t *off, const uint32_t *len, const uint32_t *addr,
             uint16_t *out, uint64_t n) {
    int dev = 0, cus = 0;
    int rc = fcs::engine_device0(&dev, &cus);
    if (rc) return rc;
    HostPipe *hp = nullptr;
    if ((rc = get_pipe(dev, cus, &hp))) return rc;
    std::lock_guard<std::mutex> lk(hp->mu);
    int cur = 0;
    HIPTRY(hipGetDevice(&cur), "hipGetDevice");
    HIPTRY(hipSetDevice(dev), "hipSetDevice");
    auto drain = [&](Slot &s) -> int {
        if (!s.live) return 0;
        HIPTRY(hipEventSynchronize(s.done), "hipEventSynchronize");
        std::memcpy(out + s.i0, s.h_out, s.n * 2);
        s.live = false;
        return 0;
    };
    uint64_t i = 0;
    int b = 0;
    auto step = [&]() -> int {
        Slot &s = hp->slot[b];
        int rc = drain(s);
        if (rc) return rc;
        // the chunk [i, e): at most kChunkPkts packets, kChunkBytes of packet bytes, and (so that
        // densely packed packets go over as one span copy) a span of at most kChunkBytes unless
        // the packets are sparse (span > 2x their bytes), which are gathered instead
        uint64_t e = i, sum = 0, lo = UINT64_MAX, hi = 0;
        while (e < n && e - i < kChunkPkts && sum + len[e] <= kChunkBytes) {
            const uint64_t nlo = std::min(lo, off[e]), nhi = std::max(hi, off[e] + len[e]);
            if (e > i && nhi - nlo > kChunkBytes && nhi - nlo <= 2 * (sum + len[e])) break;
            sum += len[e];
            lo = nlo;
            hi = nhi;
            e++;
        }
        if (e == i)
            return fcs::set_error(EINVAL, "packet %llu of %u bytes exceeds the %llu-byte host chunk",
                                  (unsigned long long)i, len[i], (unsigned long long)kChunkBytes);
        const uint64_t np = e - i;
        uint64_t span;
        if (hi - lo <= kChunkBytes) {   // dense: one span copy, offsets rebased (alignment kept mod 16)
            const uint64_t pad = lo & 15;
            span = pad + (hi - lo);
            fcs::staging_copy(s.h_in + pad, arena + lo, hi - lo);
            for (uint64_t q = 0; q < np; q++) s.h_off[q] = off[i + q] - lo + pad;
        } else {                        // sparse: gather back to back (any start alignment is fine)
            uint64_t w = 0;
            for (uint64_t q = 0; q < np; q++) {
                const uint64_t a = off[i + q];
                std::memcpy(s.h_in + w, arena + a, len[i + q]);
                s.h_off[q] = w;
                w += len[i + q];
            }
            span = w;
        }
        std::memcpy(s.h_len, len + i, np * 4);
        if (addr) std::memcpy(s.h_addr, addr + 2 * i, np * 8);
        hipStream_t st = hp->stream;
        HIPTRY(hipMemcpyAsync(s.d_in, s.h_in, span, hipMemcpyHostToDevice, st), "H2D packets");
        HIPTRY(hipMemcpyAsync(s.d_off, s.h_off, np * 8, hipMemcpyHostToDevice, st), "H2D off");
        HIPTRY(hipMemcpyAsync(s.d_len, s.h_len, np * 4, hipMemcpyHostToDevice, st), "H2D len");
        if (addr) HIPTRY(hipMemcpyAsync(s.d_addr, s.h_addr, np * 8, hipMemcpyHostToDevice, st), "H2D addr");
        inet::IParams p{};
        p.base = (uint64_t)s.d_in;
        p.off = s.d_off;
        p.len = s.d_len;
        p.addr = addr ? s.d_addr : nullptr;
        p.out = s.d_out;
        p.n = np;
        if ((rc = launch_counted(true, mode, p, hp->dev, cus, st))) return rc;
        HIPTRY(hipMemcpyAsync(s.h_out, s.d_out, np * 2, hipMemcpyDeviceToHost, st), "D2H checksums");
        HIPTRY(hipEventRecord(s.done, st), "hipEventRecord");
        s.live = true;
        s.i0 = i;
        s.n = np;
        i = e;
        b = (b + 1) % kDepth;
        return 0;
    };
    while (i < n && !rc) rc = step();
    if (rc) {   // never leave a slot that would later be drained into this call's `out`
        (void)hipStreamSynchronize(hp->stream);
        for (Slot &s : hp->slot) s.live = false;
    }
    for (Slot &s : hp->slot) {
        const int r2 = drain(s);
        if (!rc) rc = r2;
    }
    hipSetDevice(cur);
    return rc;
}

uint16_t single_or_die(int mode, const void *dp, size_t bsize, uint32_t src, uint32_t dst, const char *name) {
    if (bsize > UINT32_MAX) {
        std::fprintf(stderr, "nstack_fcs: %s: %zu-byte packet exceeds the engine's 32-bit length\n", name, bsize);
        std::abort();
    }
    const uint64_t off = 0;
    const uint32_t len = (uint32_t)bsize, addr[2] = {src, dst};
    uint16_t out = 0;
    static const uint8_t kEmpty[1] = {0};
    const int rc = run_host(mode, bsize ? (const uint8_t *)dp : kEmpty, &off, &len, addr, &out, 1);
    if (rc) {
        std::fprintf(stderr, "nstack_fcs: %s: no usable GPU engine: %s\n", name, fcs_last_error());
        std::abort();
    }
    return out;
}

}  // namespace

extern "C" {

int inet_csum_batch_dev(int mode, const void *arena, uint64_t arena_bytes, const uint64_t *off,
                        const uint32_t *len, const uint32_t *addr, uint16_t *out, uint64_t n, void *stream) {
    int rc = check_mode(mode, addr);
    if (rc || n == 0) return rc;
    if (!arena || !off || !len || !out) return fcs::set_error(EINVAL, "null pointer");
    (void)arena_bytes;   // device arrays: bounds are the caller's contract (as ether_fcs_batch_dev)
    int dev = 0, cus = 0;
    if ((rc = fcs::current_device(&dev, &cus))) return rc;
    inet::IParams p{};
    p.base = (uint64_t)arena;
    p.off = off;
    p.len = len;
    p.addr = addr;
    p.out = out;
    p.n = n;
    return launch_counted(true, mode, p, dev, cus, (hipStream_t)stream);
}

int inet_csum_fixed_dev(int mode, const void *base, uint64_t stride, uint32_t len, uint64_t n,
                        const uint32_t *addr, uint16_t *out, void *stream) {
    int rc = check_mode(mode, addr);
    if (rc || n == 0) return rc;
    if (!base || !out) return fcs::set_error(EINVAL, "null pointer");
    if (n > 1 && stride < len) return fcs::set_error(EINVAL, "stride %llu < len %u", (unsigned long long)stride, len);
    int dev = 0, cus = 0;
    if ((rc = fcs::current_device(&dev, &cus))) return rc;
    inet::IParams p{};
    p.base = (uint64_t)base;
    p.stride = stride;
    p.flen = len;
    p.addr = addr;
    p.out = out;
    p.n = n;
    return launch_counted(false, mode, p, dev, cus, (hipStream_t)stream);
}

int inet_csum_batch_host(int mode, const void *arena, uint64_t arena_bytes, const uint64_t *off,
                         const uint32_t *len, const uint32_t *addr, uint16_t *out, uint64_t n) {
    int rc = check_mode(mode, addr);
    if (rc || n == 0) return rc;
    if (!arena || !off || !len || !out) return fcs::set_error(EINVAL, "null pointer");
    for (uint64_t i = 0; i < n; i++)
        if (off[i] > arena_bytes || len[i] > arena_bytes - off[i])
            return fcs::set_error(EINVAL, "packet %llu [%llu, +%u) outside the %llu-byte arena",
                                  (unsigned long long)i, (unsigned long long)off[i], len[i],
                                  (unsigned long long)arena_bytes);
    return run_host(mode, (const uint8_t *)arena, off, len, addr, out, n);
}

uint64_t inet_csum_set_flat_threshold(uint64_t packets) { return g_flat_min.exchange(packets); }

uint64_t inet_csum_set_dma_threshold(uint64_t packets) { return g_dma_min.exchange(packets); }

uint16_t inet_ip_checksum(const void *dp, size_t bsize) {
    return single_or_die(INET_CSUM_IP, dp, bsize, 0, 0, "inet_ip_checksum");
}

uint16_t inet_tcp_checksum(uint32_t src, uint32_t dst, const void *dp, size_t bsize) {
    return single_or_die(INET_CSUM_TCP, dp, bsize, src, dst, "inet_tcp_checksum");
}

uint16_t inet_udp_checksum(const void *dp, size_t len, uint32_t src, uint32_t dst) {
    return single_or_die(INET_CSUM_UDP, dp, len, src, dst, "inet_udp_checksum");
}

}  // extern "C"
