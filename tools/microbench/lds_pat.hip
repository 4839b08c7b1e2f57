// lds_pat.hip — LDS read cost per wave-instruction for given per-lane address patterns (measurement
// probe for the flat kernel's slot layout). Every CU runs W waves; each wave issues
// ITER x 8 independent ds_read_b32 or ds_read_b128 at (pattern offset of its lane) + 8 KiB * k and
// waits; s_memtime (shader clock) brackets the loop. Prints cycles per wave-instruction per CU
// (loop cycles / (ITER * 8 * W)): with the LDS saturated this is its issue cost for the pattern.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_pat tools/microbench/lds_pat.hip && /tmp/lds_pat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <string>

constexpr int ITER = 2048;
struct Pat { uint32_t off[64]; };

template <bool WIDE>
__global__ __launch_bounds__(1024) void probe(Pat pat, unsigned long long *cyc, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[16384];   // 64 KiB
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t a = (uint32_t)(uintptr_t)lds + pat.off[threadIdx.x & 63];
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
        if (WIDE) {
            __attribute__((ext_vector_type(4))) uint32_t v0, v1, v2, v3, v4, v5, v6, v7;
            asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(v0) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(v1) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:16384" : "=v"(v2) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:24576" : "=v"(v3) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:32768" : "=v"(v4) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:40960" : "=v"(v5) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:49152" : "=v"(v6) : "v"(a));
            asm volatile("ds_read_b128 %0, %1 offset:57344" : "=v"(v7) : "v"(a));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc ^= v0.x ^ v1.y ^ v2.z ^ v3.w ^ v4.x ^ v5.y ^ v6.z ^ v7.w;
        } else {
            uint32_t v0, v1, v2, v3, v4, v5, v6, v7;
            asm volatile("ds_read_b32 %0, %1 offset:0" : "=v"(v0) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:8192" : "=v"(v1) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:16384" : "=v"(v2) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:24576" : "=v"(v3) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:32768" : "=v"(v4) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:40960" : "=v"(v5) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:49152" : "=v"(v6) : "v"(a));
            asm volatile("ds_read_b32 %0, %1 offset:57344" : "=v"(v7) : "v"(a));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc ^= v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) atomicMax(&cyc[blockIdx.x], (unsigned long long)(t1 - t0));
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    std::vector<std::pair<std::string, std::vector<uint32_t>>> pats;
    auto add = [&](const char *name, auto f) {
        std::vector<uint32_t> o(64);
        for (int l = 0; l < 64; l++) o[l] = f(l) % 8192u;
        pats.push_back({name, o});
    };
    srand(7);
    std::vector<uint32_t> rnd(64);
    for (auto &x : rnd) x = (uint32_t)(rand() % 512) * 16u;
    add("lane*16", [](int l) { return 16u * l; });
    add("lane*32", [](int l) { return 32u * l; });
    add("lane*64", [](int l) { return 64u * l; });
    add("lane*128", [](int l) { return 128u * l; });
    add("lane*96", [](int l) { return 96u * l; });
    add("lane*4", [](int l) { return 4u * l; });
    add("lane*8", [](int l) { return 8u * l; });
    add("broadcast", [](int) { return 0u; });
    add("random16", [&](int l) { return rnd[l]; });
    add("8lanes/128B-row", [](int l) { return 16u * (l & 7) + 128u * (l >> 3); });
    add("lane*64 xor-swz", [](int l) { uint32_t b = 4u * l; return 16u * (b ^ ((b >> 3) & 7)); });
    add("lane*96 xor-swz", [](int l) { uint32_t b = 6u * l; return 16u * (b ^ ((b >> 3) & 7)); });
    add("lane*16 pairs-same", [](int l) { return 16u * (l >> 1); });
    add("half0=half1", [](int l) { return 16u * (l & 31); });
    add("quads 64B apart", [](int l) { return 16u * (l & 3) + 256u * (l >> 2); });
    unsigned long long *cyc;
    uint32_t *sink;
    const int G = 256;
    hipMalloc(&cyc, G * 8);
    hipMalloc(&sink, 4);
    for (int W : {4, 16}) {
        for (int wide = 0; wide < 2; wide++) {
            for (auto &pp : pats) {
                Pat p;
                for (int l = 0; l < 64; l++) p.off[l] = wide ? pp.second[l] & ~15u : pp.second[l] & ~3u;
                hipMemset(cyc, 0, G * 8);
                if (wide) hipLaunchKernelGGL(probe<true>, dim3(G), dim3(64 * W), 0, 0, p, cyc, sink);
                else hipLaunchKernelGGL(probe<false>, dim3(G), dim3(64 * W), 0, 0, p, cyc, sink);
                if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
                std::vector<unsigned long long> h(G);
                hipMemcpy(h.data(), cyc, G * 8, hipMemcpyDeviceToHost);
                double m = 0;
                for (auto v : h) m += (double)v;
                m /= G;
                printf("{\"waves\": %d, \"op\": \"%s\", \"pattern\": \"%s\", \"cycles_per_inst_per_cu\": %.3f}\n", W,
                       wide ? "ds_read_b128" : "ds_read_b32", pp.first.c_str(), m / (ITER * 8.0 * W));
            }
        }
    }
    return 0;
}
