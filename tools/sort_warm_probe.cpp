// Probe: wall time of the first hipcub segmented radix sort in a process against later ones
// (the cold build's target preparation showed an 8.4 ms gap before its first sort kernel).
// Build: hipcc --offload-arch=gfx950 -O2 tools/sort_warm_probe.cpp -o tools/sort_warm_probe
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <chrono>
#include <cstdio>
#include <vector>

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

static int run(int nseg, int big, const char* tag) {
    std::vector<unsigned> off(nseg + 1);
    unsigned n = 0;
    for (int i = 0; i < nseg; i++) {
        off[i] = n;
        n += (i == 0) ? (unsigned)big : 1u + (unsigned)(i % 37);
    }
    off[nseg] = n;
    float *k0, *k1;
    unsigned *v0, *v1, *o;
    hipMalloc(&k0, 4 * (size_t)n);
    hipMalloc(&k1, 4 * (size_t)n);
    hipMalloc(&v0, 4 * (size_t)n);
    hipMalloc(&v1, 4 * (size_t)n);
    hipMalloc(&o, 4 * (size_t)(nseg + 1));
    hipMemcpy(o, off.data(), 4 * (size_t)(nseg + 1), hipMemcpyHostToDevice);
    hipMemset(k0, 0, 4 * (size_t)n);
    size_t tb = 0;
    hipcub::DeviceSegmentedRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, (int)n, nseg, o, o + 1, 0, 32, 0);
    void* tmp;
    hipMalloc(&tmp, tb + 16);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 3; rep++) {
        const auto t0 = std::chrono::steady_clock::now();
        hipError_t e = hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, (int)n, nseg, o,
                                                                  o + 1, 0, 32, 0);
        const double call = ms_since(t0);
        hipDeviceSynchronize();
        printf("%s rep %d: n %u segs %d  call %.3f ms  call+sync %.3f ms  err %d\n", tag, rep, n, nseg,
               call, ms_since(t0), (int)e);
    }
    hipFree(k0); hipFree(k1); hipFree(v0); hipFree(v1); hipFree(o); hipFree(tmp);
    return 0;
}

int main() {
    const auto t0 = std::chrono::steady_clock::now();
    hipFree(nullptr);
    printf("init %.3f ms\n", ms_since(t0));
    run(4, 5000, "tiny");
    run(1000000, 200000, "c4-like");
    return 0;
}
