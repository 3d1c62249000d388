// Shared host-side helpers of libmetacov_amd (error state, checks).
#pragma once

#include <cstdarg>
#include <cstdio>
#include <string>

namespace mc {

// Thread-local message of the last error (mc_last_error()).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* last_error();

}  // namespace mc

#define MC_REQUIRE(cond, code, ...)        \
    do {                                   \
        if (!(cond)) {                     \
            mc::set_error(__VA_ARGS__);    \
            return (code);                 \
        }                                  \
    } while (0)
