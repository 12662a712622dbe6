// topo_dev_common.h -- device helpers shared by the SSSP kernels (topo_kernels.hip,
// topo_sssp_batch.hip): f64 bit views, L1-bypassing loads, the 12-B adjacency record,
// wave-level reductions and wave-aggregated queue appends.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "topo_device.h"

namespace shdtopo {
namespace dev {

constexpr unsigned long long kInfBits = 0x7FF0000000000000ull;

__device__ __forceinline__ unsigned long long ld_l2_u64(const unsigned long long* p) {
    // L1-bypassing (sc1) load: values written by atomics of other waves must not be read from a
    // stale vector-L1 line (MI355X_MICROARCH.md "inter-workgroup visibility").
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_l2_u32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double bits2d(unsigned long long b) {
    return __longlong_as_double((long long)b);
}
__device__ __forceinline__ unsigned long long d2bits(double d) {
    return (unsigned long long)__double_as_longlong(d);
}

// adjacency record, 16 B (one aligned 16-B load): a = neighbour (column), p = f32 bits of
// pi(a) = d(h0, a) rounded up (the landmark bound of the batch kernel's relaxation filter),
// (b, c) = the f64 edge latency (low, high word)
struct __attribute__((aligned(16))) AdjRec {
    uint32_t a, p, b, c;
};
constexpr unsigned long long kAdjWords = 4;
__device__ __forceinline__ uint32_t adj_col(const DevCSR& g, uint32_t j) {
    return g.adj[kAdjWords * j];
}
__device__ __forceinline__ const AdjRec& adj_rec(const DevCSR& g, uint32_t j) {
    return *reinterpret_cast<const AdjRec*>(g.adj + kAdjWords * j);
}
__device__ __forceinline__ void adj_load(const DevCSR& g, uint32_t j, uint32_t& col, double& wt) {
    const AdjRec r = adj_rec(g, j);
    col = r.a;
    wt = __hiloint2double((int)r.c, (int)r.b);
}
__device__ __forceinline__ double rec_wt(const AdjRec& r) {
    return __hiloint2double((int)r.c, (int)r.b);
}

// Bucket of a distance: floor(x / delta) by one IEEE multiply, monotone non-decreasing in x (so a
// bucket is an interval of distances); +inf and huge values land in the last bucket.
__device__ __forceinline__ uint32_t bucket_of(double x, double inv_delta) {
    const double b = x * inv_delta;
    return b < 4.0e9 ? (uint32_t)b : 4000000000u;
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    return x;
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    return x;
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// Block-wide exclusive scan of one u32 per thread (NT threads, NT/64 words of LDS scratch in
// `wave`); *total receives the sum.  Contains barriers: every thread must call it.
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, uint32_t* wave, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NW = NT / 64;
    uint32_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) wave[wid] = v;
    __syncthreads();
    if (wid == 0) {
        uint32_t w = lane < NW ? wave[lane] : 0u;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            uint32_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < NW) wave[lane] = w;
    }
    __syncthreads();
    uint32_t base = wid ? wave[wid - 1] : 0u;
    *total = wave[NW - 1];
    __syncthreads();
    return base + v - x;
}

// Wave-aggregated queue append of one value per predicated lane: one LDS atomic per wave.  A push
// past `cap` is dropped and ORs `code` into *lds_over.
template <class T>
__device__ __forceinline__ void wave_push_t(bool pred, T val, T* q, uint32_t* lds_tail,
                                            uint32_t cap, uint32_t* lds_over, uint32_t code) {
    unsigned long long m = __ballot(pred);
    if (m == 0ull) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(lds_tail, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) {
        const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (pos < cap) q[pos] = val;
        else atomicOr(lds_over, code);
    }
}

}  // namespace dev
}  // namespace shdtopo
