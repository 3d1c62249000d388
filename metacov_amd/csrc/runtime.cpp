// mc_runtime_init (include/metacov_amd.h): the HIP runtime and one device's
// context, queues and allocators brought up ahead of the first mc_ctx, so a
// caller can overlap that start-up with its own (the CLI: with Python's
// imports, on a thread).  Everything it creates is released again; what
// stays is the runtime's own state (the device context, its hardware queues,
// the allocators' pools), which the first mc_ctx_create then finds ready.
#include <hip/hip_runtime.h>

#include "../../include/metacov_amd.h"
#include "common.h"

extern "C" int mc_runtime_init(int device) {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    MC_REQUIRE(e == hipSuccess && n > 0, MC_E_HIP, "no HIP device available (hipGetDeviceCount: %s)",
               hipGetErrorString(e));
    if (device < 0 || device >= n) return MC_OK;   // the runtime only
    if (hipSetDevice(device) != hipSuccess || hipFree(nullptr) != hipSuccess) {
        mc::set_error("hipSetDevice(%d) failed", device);
        return MC_E_HIP;
    }
    hipStream_t s = nullptr;   // a stream's first creation sets up the device's hardware queues
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) {
        void* d = nullptr;
        void* h = nullptr;
        if (hipMalloc(&d, 256) == hipSuccess) (void)hipFree(d);
        if (hipHostMalloc(&h, 4096, hipHostMallocDefault) == hipSuccess) (void)hipHostFree(h);
        hipEvent_t ev = nullptr;
        if (hipEventCreate(&ev) == hipSuccess) {
            (void)hipEventRecord(ev, s);
            (void)hipEventSynchronize(ev);
            (void)hipEventDestroy(ev);
        }
        (void)hipStreamDestroy(s);
    }
    (void)hipGetLastError();
    return MC_OK;
}
