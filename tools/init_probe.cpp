// Probe: what a process's first HIP calls cost (dev_init of the routing engine): device count,
// set device, context (hipFree(0)), the first and second stream, a malloc, a memset.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
int main() {
    auto t = std::chrono::steady_clock::now();
    auto mark = [&](const char* w) {
        auto n = std::chrono::steady_clock::now();
        printf("%-28s %8.2f ms\n", w, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    };
    int n = 0;
    (void)hipGetDeviceCount(&n); mark("hipGetDeviceCount");
    (void)hipSetDevice(0); mark("hipSetDevice");
    (void)hipFree(nullptr); mark("hipFree(0)");
    void* p = nullptr;
    (void)hipMalloc(&p, 1 << 20); mark("hipMalloc 1 MiB");
    hipStream_t s1, s2, s3;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking); mark("stream 1 (non-blocking)");
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking); mark("stream 2 (non-blocking)");
    (void)hipStreamCreate(&s3); mark("stream 3 (default flags)");
    (void)hipMemsetAsync(p, 0, 1 << 20, s1); (void)hipStreamSynchronize(s1); mark("memset on stream 1");
    (void)hipMemsetAsync(p, 0, 1 << 20, nullptr); (void)hipDeviceSynchronize(); mark("memset on null stream");
    return 0;
}
