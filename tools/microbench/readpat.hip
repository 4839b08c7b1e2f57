// Read-pattern microbenchmark for the FCS kernel layout decision (not product code).
// Measures HBM read GB/s of: (1) a coalesced 16 B/lane stream, (2) the 48 B/lane
// half-wave-per-1518B-frame chunk layout at 4-byte alignment (3 x dwordx4 + dword),
// (3) the same layout with 16-byte-aligned 64 B windows.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream(const u32x4* __restrict__ p, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  for (; i + 3 * st < n16; i += 4 * st) {
    u32x4 a = p[i], b = p[i + st], c = p[i + 2 * st], d = p[i + 3 * st];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += st) { u32x4 a = p[i]; acc ^= a.x ^ a.y ^ a.z ^ a.w; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_chunk(const uint8_t* __restrict__ base, size_t nframes, uint32_t L, uint32_t* out) {
  const int lane = threadIdx.x & 63, j = lane & 31, half = lane >> 5;
  size_t hw = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 32;
  size_t H = (size_t)gridDim.x * blockDim.x / 32;
  uint32_t acc = 0;
  for (size_t f = hw; f < nframes; f += H) {
    uint64_t end = (uint64_t)base + f * L + L;
    uint64_t cs = end - 48 * (j + 1);
    if (cs < (uint64_t)base) cs = (uint64_t)base;
    if (MODE == 0) {
      const u32x4a4* q = (const u32x4a4*)(cs & ~3ull);
      u32x4a4 a = q[0], b = q[1], c = q[2];
      uint32_t d = ((const uint32_t*)q)[12];
      acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d;
    } else {
      const u32x4* q = (const u32x4*)(cs & ~15ull);
      u32x4 a = q[0], b = q[1], c = q[2], d = q[3];
      acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ half;
}

int main(int argc, char** argv) {
  size_t nframes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 20);
  uint32_t L = 1518;
  size_t bytes = nframes * L + 64;
  uint8_t* buf; uint32_t* out;
  CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&out, 1 << 26));
  CK(hipMemset(buf, 0x5a, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int grids[] = {1024, 2048, 4096, 8192};
  for (int mode = 0; mode < 3; mode++) {
    for (int g : grids) {
      float best = 1e9, tot = 0;
      for (int r = 0; r < 6; r++) {
        CK(hipEventRecord(e0));
        if (mode == 0) k_stream<<<g, 256>>>((const u32x4*)buf, (nframes * L) / 16, out);
        else if (mode == 1) k_chunk<0><<<g, 256>>>(buf, nframes, L, out);
        else k_chunk<1><<<g, 256>>>(buf, nframes, L, out);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) { best = ms < best ? ms : best; tot += ms; }
      }
      double gb = (double)nframes * L / 1e9;
      printf("mode=%d grid=%d best=%.3f ms  %.1f GB/s (best)  %.1f GB/s (mean)\n", mode, g, best, gb / best * 1e3, gb / (tot / 5) * 1e3);
    }
  }
  CK(hipGetLastError());
  return 0;
}
