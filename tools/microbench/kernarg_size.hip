// kernarg_size.hip — does a launch with large by-value kernel arguments work on this stack?
// (measurement probe: sums a 2/4/8/16 KiB argument array on the device and compares).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int N> struct Big { uint32_t w[N]; };
template <int N> __global__ void sum_kernel(Big<N> a, unsigned long long *out) {
    unsigned long long s = 0;
    for (int i = threadIdx.x; i < N; i += 64) s += a.w[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (threadIdx.x == 0) *out = s;
}
template <int N> int probe() {
    Big<N> a;
    unsigned long long want = 0;
    for (int i = 0; i < N; i++) { a.w[i] = i * 2654435761u; want += a.w[i]; }
    unsigned long long *d, got = 0;
    if (hipMalloc(&d, 8) != hipSuccess) return 1;
    hipMemset(d, 0, 8);
    hipLaunchKernelGGL(sum_kernel<N>, dim3(1), dim3(64), 0, 0, a, d);
    hipError_t e = hipGetLastError();
    hipError_t s = hipDeviceSynchronize();
    hipMemcpy(&got, d, 8, hipMemcpyDeviceToHost);
    printf("{\"arg_bytes\": %d, \"launch\": \"%s\", \"sync\": \"%s\", \"ok\": %s}\n", N * 4, hipGetErrorString(e),
           hipGetErrorString(s), got == want ? "true" : "false");
    hipFree(d);
    return 0;
}
int main() { probe<512>(); probe<1024>(); probe<2048>(); probe<4096>(); return 0; }
