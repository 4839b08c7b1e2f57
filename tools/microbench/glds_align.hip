// glds_align.hip — does global_load_lds_dwordx4 (LDS-DMA, 16 B per lane) honour global addresses
// that are 4-byte but not 16-byte aligned? (measurement probe for a flat-kernel variant that would
// DMA each lane's own unaligned 96-B window) One wave: lane l loads 16 bytes from
// src + off + 100 l into LDS at 16 l; the wave then copies the LDS back out and the host compares
// with the source bytes, for off = 0, 4, 8, 12 (and 1, 2: byte offsets, for the record).
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/glds_align tools/microbench/glds_align.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ __launch_bounds__(64) void probe(const uint8_t *src, uint32_t off, uint8_t *dst) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[1024];
    typedef __attribute__((address_space(3))) void lds_void;
    const int lane = threadIdx.x;
    for (int i = lane; i < 256; i += 64) reinterpret_cast<uint32_t *>(lds)[i] = 0xDEADBEEFu;
    __syncthreads();
    const uint8_t *g = src + off + 100u * (uint32_t)lane;
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(g), (lds_void *)lds, 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    __syncthreads();
    for (int i = 0; i < 16; i++) dst[16 * lane + i] = lds[16 * lane + i];
}

int main() {
    const size_t n = 8192;
    std::vector<uint8_t> h(n);
    for (size_t i = 0; i < n; i++) h[i] = (uint8_t)(i * 131 + 7);
    uint8_t *src, *dst;
    if (hipMalloc(&src, n) != hipSuccess || hipMalloc(&dst, 1024) != hipSuccess) return 1;
    hipMemcpy(src, h.data(), n, hipMemcpyHostToDevice);
    for (uint32_t off : {0u, 4u, 8u, 12u, 1u, 2u}) {
        hipMemset(dst, 0, 1024);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, off, dst);
        if (hipDeviceSynchronize() != hipSuccess) {
            printf("{\"off\": %u, \"launch\": \"failed\"}\n", off);
            return 1;
        }
        std::vector<uint8_t> o(1024);
        hipMemcpy(o.data(), dst, 1024, hipMemcpyDeviceToHost);
        int bad = 0, first = -1;
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 16; i++)
                if (o[16 * l + i] != h[off + 100 * l + i]) {
                    bad++;
                    if (first < 0) first = 16 * l + i;
                }
        // what a 16-B-aligned fetch of the same lane would give, for diagnosis
        int as_floor16 = 0;
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 16; i++)
                if (o[16 * l + i] == h[((off + 100 * l) & ~15u) + i]) as_floor16++;
        printf("{\"off\": %u, \"bytes_wrong\": %d, \"first_wrong\": %d, \"bytes_matching_floor16_fetch\": %d}\n", off, bad,
               first, as_floor16);
    }
    return 0;
}
