// fcs_error.hpp — error reporting shared by the library's translation units (not exported).
#pragma once

namespace fcs {
// Records the message for fcs_last_error() (per thread) and returns -err.
__attribute__((visibility("hidden"))) int set_error(int err, const char *fmt, ...)
    __attribute__((format(printf, 2, 3)));
}  // namespace fcs
