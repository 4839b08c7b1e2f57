// wave_sync.hpp — ordering for lanes of one wave that hand values to each other through LDS.
#pragma once
#include <hip/hip_runtime.h>

// Lanes of one wave handing values to each other through LDS (frame-start marks, frame lists,
// accumulators) race under the HIP memory model unless the write and the other lanes' read are
// ordered, and the compiler does exploit it: it moved a lane's read of mark[lane] into the branch
// where that lane itself writes a mark. A wavefront-scope release fence, a wave
// barrier and an acquire fence order every LDS write before it with every LDS access after it.
__device__ __forceinline__ void wave_lds_sync() {
#ifndef FCS_NO_WAVE_SYNC   // measurement-only: the unordered form (racy; timing comparison only)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}
