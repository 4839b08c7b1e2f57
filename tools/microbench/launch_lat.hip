// launch_lat.hip — small-batch latency floor on one MI355X (measurement tool): host round trip of
//   (a) an empty kernel + hipStreamSynchronize,
//   (b) an empty kernel that writes a flag into host-mapped memory, host spinning on the flag,
//   (c) as (b) but the kernel first stages 148 KiB of tables into LDS (what every FCS launch does),
//   (d) the resident-kernel hand-off: a kernel polling a doorbell in host memory, host spinning on
//       its completion flag (no launch per job).
// Build: hipcc --offload-arch=gfx950 -O2 tools/microbench/launch_lat.hip -o tools/microbench/launch_lat
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

__global__ void k_empty() {}
__global__ void k_flag(volatile uint64_t *flag, uint64_t v) {
    if (threadIdx.x == 0) __hip_atomic_store((uint64_t *)flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ __launch_bounds__(1024) void k_stage_flag(const uint32_t *blob, volatile uint64_t *flag, uint64_t v) {
    __shared__ uint32_t lds[37888];
    for (int i = threadIdx.x; i < 37888; i += 1024) lds[i] = blob[i & 8191];
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((uint64_t *)flag, v + lds[v & 1023] * 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_resident(uint64_t *door, uint64_t *done, uint64_t n) {
    if (threadIdx.x != 0) return;
    uint64_t last = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (last < n) {
        uint64_t d;
        while ((d = __hip_atomic_load(door, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) == last) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) return;   // 5 s: never outlive the host
            __builtin_amdgcn_s_sleep(1);
        }
        last = d;
        __hip_atomic_store(done, d, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double us_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    uint64_t *h;
    hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
    uint64_t *d;
    hipHostGetDevicePointer((void **)&d, h, 0);
    uint32_t *blob;
    hipMalloc(&blob, 8192 * 4);
    hipMemset(blob, 0, 8192 * 4);
    const int N = 2000;
    auto t = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); hipStreamSynchronize(st); }
    t = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); hipStreamSynchronize(st); }
    printf("{\"path\": \"empty+sync\", \"us\": %.2f}\n", us_since(t) / N);
    h[0] = 0;
    t = std::chrono::steady_clock::now();
    for (int i = 1; i <= N; i++) {
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, (volatile uint64_t *)d, (uint64_t)i);
        auto w = std::chrono::steady_clock::now();
        while (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) != (uint64_t)i)
            if (us_since(w) > 1e6) { printf("flag never arrived\n"); return 1; }
    }
    printf("{\"path\": \"empty+flag spin\", \"us\": %.2f}\n", us_since(t) / N);
    hipStreamSynchronize(st);
    h[0] = 0;
    t = std::chrono::steady_clock::now();
    for (int i = 1; i <= N; i++) {
        hipLaunchKernelGGL(k_stage_flag, dim3(1), dim3(1024), 0, st, blob, (volatile uint64_t *)d, (uint64_t)i);
        auto w = std::chrono::steady_clock::now();
        while (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) != (uint64_t)i)
            if (us_since(w) > 1e6) { printf("flag never arrived\n"); return 1; }
    }
    printf("{\"path\": \"148KiB LDS staging+flag spin\", \"us\": %.2f}\n", us_since(t) / N);
    hipStreamSynchronize(st);
    h[1] = 0; h[2] = 0;
    hipLaunchKernelGGL(k_resident, dim3(1), dim3(64), 0, st, d + 1, d + 2, (uint64_t)N);
    t = std::chrono::steady_clock::now();
    for (int i = 1; i <= N; i++) {
        __atomic_store_n(&h[1], (uint64_t)i, __ATOMIC_RELEASE);
        auto w = std::chrono::steady_clock::now();
        while (__atomic_load_n(&h[2], __ATOMIC_ACQUIRE) != (uint64_t)i) {
            if (us_since(w) > 1e6) { printf("resident kernel stuck\n"); return 1; }
        }
    }
    printf("{\"path\": \"resident doorbell round trip\", \"us\": %.2f}\n", us_since(t) / N);
    hipStreamSynchronize(st);
    return 0;
}
