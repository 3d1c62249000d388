// Can the GPU DMA straight from the page cache?  A read-only shared mapping of
// a file registered with hipHostRegister (hipHostRegisterReadOnly), then
// copied up, against the pread-into-pinned-staging path the GPU decode uses.
//   hostreg_probe FILE [slice_MiB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>
#include <atomic>
#include <thread>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                          \
            return 1;                                                               \
        }                                                                           \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const size_t slice = (size_t)(argc > 2 ? atoi(argv[2]) : 256) << 20;
    int fd = open(argv[1], O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    const size_t n = (size_t)st.st_size;
    uint8_t* d = nullptr;
    CK(hipMalloc(&d, n));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // A: pread into one pinned slice at a time (single thread; the decode uses 16)
    {
        uint8_t* h = nullptr;
        CK(hipHostMalloc(&h, slice, 0));
        double t0 = now();
        for (size_t at = 0; at < n; at += slice) {
            const size_t m = std::min(slice, n - at);
            size_t got = 0;
            while (got < m) got += pread(fd, h + got, m - got, at + got);
            CK(hipMemcpyAsync(d + at, h, m, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
        }
        printf("pread+pinned (1 thread, serial): %.1f ms  %.1f GB/s\n", (now() - t0) * 1e3, n / (now() - t0) / 1e9);
        CK(hipHostFree(h));
    }
    // B: register slices of a shared read-only mapping, copy from them
    void* m = mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) {
        printf("mmap failed\n");
        return 1;
    }
    double treg = 0, tcopy = 0, tunreg = 0;
    const double t0 = now();
    for (size_t at = 0; at < n; at += slice) {
        const size_t len = std::min(slice, n - at);
        double a = now();
        hipError_t e = hipHostRegister((uint8_t*)m + at, len, hipHostRegisterReadOnly);
        if (e != hipSuccess) {
            printf("hipHostRegister(ReadOnly) failed at %zu: %s\n", at, hipGetErrorString(e));
            (void)hipGetLastError();
            e = hipHostRegister((uint8_t*)m + at, len, hipHostRegisterDefault);
            printf("hipHostRegister(Default): %s\n", hipGetErrorString(e));
            if (e != hipSuccess) return 1;
        }
        double b = now();
        CK(hipMemcpyAsync(d + at, (uint8_t*)m + at, len, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double c = now();
        CK(hipHostUnregister((uint8_t*)m + at));
        double e2 = now();
        treg += b - a;
        tcopy += c - b;
        tunreg += e2 - c;
    }
    const double tt = now() - t0;
    printf("register+copy+unregister: %.1f ms (register %.1f, copy %.1f, unregister %.1f)  %.1f GB/s\n", tt * 1e3,
           treg * 1e3, tcopy * 1e3, tunreg * 1e3, n / tt / 1e9);
    // check: the device bytes equal the file's
    std::vector<uint8_t> back(1 << 20);
    for (size_t at : {(size_t)0, n / 2, n - back.size()}) {
        CK(hipMemcpy(back.data(), d + at, back.size(), hipMemcpyDeviceToHost));
        if (memcmp(back.data(), (uint8_t*)m + at, back.size())) {
            printf("MISMATCH at %zu\n", at);
            return 1;
        }
    }
    printf("bytes equal\n");
    // C: registration on nthr threads (a queue of slices), copies in order as
    // slices become registered, unregistration after each copy
    for (int nthr : {4, 16}) {
        CK(hipMemset(d, 0, n));
        const int64_t ns = (int64_t)((n + slice - 1) / slice);
        std::vector<std::atomic<int>> ready(ns);
        for (auto& r : ready) r = 0;
        std::atomic<int64_t> next{0};
        const double tc0 = now();
        std::vector<std::thread> th;
        for (int t = 0; t < nthr; ++t)
            th.emplace_back([&]() {
                hipSetDevice(0);
                for (int64_t i; (i = next.fetch_add(1)) < ns;) {
                    const size_t at = (size_t)i * slice, len = std::min(slice, n - at);
                    ready[i] = hipHostRegister((uint8_t*)m + at, len, hipHostRegisterReadOnly) == hipSuccess ? 1 : -1;
                }
            });
        bool ok = true;
        for (int64_t i = 0; i < ns; ++i) {
            while (ready[i].load() == 0) std::this_thread::yield();
            if (ready[i] < 0) { ok = false; continue; }
            const size_t at = (size_t)i * slice, len = std::min(slice, n - at);
            CK(hipMemcpyAsync(d + at, (uint8_t*)m + at, len, hipMemcpyHostToDevice, s));
        }
        CK(hipStreamSynchronize(s));
        const double tc = now() - tc0;
        for (auto& t : th) t.join();
        for (int64_t i = 0; i < ns; ++i)
            if (ready[i] > 0) (void)hipHostUnregister((uint8_t*)m + (size_t)i * slice);
        printf("%d register threads, copies in order: %.1f ms  %.1f GB/s  %s\n", nthr, tc * 1e3, n / tc / 1e9,
               ok ? "" : "(some registrations failed)");
    }
    munmap(m, n);
    close(fd);
    return 0;
}
