// fcs_device.hpp — device lookup shared by the library's translation units (not exported).
#pragma once
#include <stdint.h>

namespace fcs {
// The calling thread's current HIP device, checked to be a gfx950 (lazily initialised engine
// state). Returns 0 or -errno (with fcs_last_error() set).
__attribute__((visibility("hidden"))) int current_device(int *dev, int *cus);
// The first device of the engine's device set (fcs_engine_init), for the host entry points.
__attribute__((visibility("hidden"))) int engine_device0(int *dev, int *cus);
// memcpy into pinned staging, split over a few threads for large spans (host pipelines).
__attribute__((visibility("hidden"))) void staging_copy(uint8_t *dst, const uint8_t *src, uint64_t bytes);
}  // namespace fcs
