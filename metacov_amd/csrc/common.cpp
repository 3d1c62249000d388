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
extern "C" const char* mc_version(void) { return "metacov_amd 0.1.0 (gfx950)"; }
