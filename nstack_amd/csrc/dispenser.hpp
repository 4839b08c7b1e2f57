// dispenser.hpp — the work dispenser shared by the persistent kernels of fcs_kernel.hip and
// inet_kernel.hip (device code).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fcs {

// Hands out the units [0, U) of a launch to the waves of a persistent grid (wave-uniform state).
// Without a counter: wave wid of W takes wid, wid + W, ... (interleaved). With one (a zeroed device
// word, KParams::ctr): the first (100 - dyn_pct) % of the units that way, the rest in chunks of
// consecutive units from *ctr, sized by the work left (guided: left / 2W, clamped to cmin..cmax),
// each chunk requested when the previous one starts so the atomic's latency stays hidden.
struct Dispenser {
    static constexpr uint64_t kEnd = ~0ull;
    unsigned long long *ctr;
    uint64_t U, W, wid, Is, Ks;
    uint64_t k = 0, ce = 0, pend = 0, psize = 0, seen = 0;
    uint32_t cmin, cmax;
    uint32_t align = 1;   // chunks of at least `align` units are cut to multiples of it (aligned result runs)
    int lane;
    bool dyn = false;

    __device__ Dispenser(unsigned long long *ctr_, uint64_t U_, uint64_t W_, uint64_t wid_, int lane_,
                         uint32_t dyn_pct, uint32_t cmin_, uint32_t cmax_)
        : ctr(ctr_), U(U_), W(W_), cmin(cmin_), cmax(cmax_), lane(lane_) {
        // wave-uniform by construction; said so, the compiler keeps the whole schedule in SGPRs
        // (from threadIdx.x >> 6 it kept it in VGPRs: 64-bit VALU division, and a VGPR spill in
        // the flat kernel)
        wid = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(wid_ >> 32)) << 32) |
              (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)wid_);
        Is = ctr ? (U * (100 - dyn_pct) / 100) / W * W : U;   // statically assigned units in all
        Ks = wid < Is ? (Is - wid + W - 1) / W : 0;             // ... of this wave
    }
    __device__ void grab() {
        const uint64_t left = U - Is > seen ? U - Is - seen : 0;
        uint64_t sz = left / (2 * W);
        sz = sz < cmin ? cmin : (sz > cmax ? cmax : sz);
        if (sz >= align) sz -= sz % align;
        uint64_t v = 0;
        if (lane == 0) v = atomicAdd(ctr, (unsigned long long)sz);
        pend = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
               (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
        psize = sz;
    }
    __device__ uint64_t take() {   // move to the requested chunk, request the one after it
        const uint64_t cb = Is + pend;
        seen = pend + psize;
        if (cb >= U) return kEnd;
        ce = cb + psize < U ? cb + psize : U;
        grab();
        return cb;
    }
    __device__ uint64_t first() {
        if (ctr) grab();   // the first dynamic chunk, requested while the static share runs
        if (Ks) return wid;
        if (!ctr) return kEnd;
        dyn = true;
        return take();
    }
    __device__ uint64_t next(uint64_t cur) {
        if (!dyn) {
            if (k + 1 < Ks) return wid + (++k) * W;
            if (!ctr) return kEnd;
            dyn = true;
            return take();
        }
        return cur + 1 < ce ? cur + 1 : take();
    }
};

}  // namespace fcs
