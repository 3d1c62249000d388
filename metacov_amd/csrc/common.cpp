#include "common.h"

namespace mc {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

const char* last_error() { return g_err.c_str(); }

}  // namespace mc

extern "C" const char* mc_last_error(void) { return mc::last_error(); }
extern "C" const char* mc_version(void) { return "metacov_amd 0.3.0 (gfx950)"; }

#ifndef MC_SOURCE_HASH
#define MC_SOURCE_HASH "unstamped"
#endif
// metacov_amd/build.py stamps the SHA-256 of the sources it built from
extern "C" const char* mc_build_id(void) { return "mc-source-sha256:" MC_SOURCE_HASH; }
