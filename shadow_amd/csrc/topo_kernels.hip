// topo_kernels.hip -- CDNA4 (gfx950) kernels of the routing engine besides the batched SSSP
// (topo_sssp_batch.hip), the heap replay (topo_replay.hip) and the graph preparation
// (topo_prep.hip):
//
//   pair_table_complete_kernel  replaces _topology_lookupPath (shd-topology.c:835-873).
//   packet_route_kernel         replaces worker_schedulePacket (src/engine/shd-worker.c:332-370)
//                               for a whole scheduler window.
//   row_min_kernel              row minima of a table (the lazy runahead's bookkeeping,
//                               shd-topology.c:500-511).
//
// f64 arithmetic: every latency add is a single IEEE add (built with -ffp-contract=off);
// reliability multiplies happen in the reference order.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "topo_dev_common.h"

namespace shdtopo {

using namespace dev;

// ------------------------------------------------------------------------------------------
// complete graphs: _topology_lookupPath (shd-topology.c:835-873) for every attached pair, and the
// row minima (the runahead bookkeeping, shd-topology.c:500-511) in the same launch: one workgroup
// per row (grid-stride over rows), the row's records written coalesced, its minimum reduced in
// LDS.  34 B of HBM traffic per pair (8 B lat + 8 B loss read, 16 B record + 2 B hops written).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
pair_table_complete_kernel(int A, int64_t row0, int64_t rows, const double* __restrict__ elatAA,
                           const double* __restrict__ elossAA, const double* __restrict__ vlossA,
                           double2* __restrict__ out_lr, uint16_t* __restrict__ out_hops,
                           double* __restrict__ out_rowmin, unsigned long long* __restrict__ stats) {
    __shared__ unsigned long long sm[4];
    unsigned long long gm = kInfBits;
    uint32_t nerr = 0;
    for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
        const int64_t i = row0 + r;
        const double vi = vlossA[i];
        unsigned long long m = kInfBits;
        for (int c = (int)threadIdx.x; c < A; c += 256) {
            const double el = elatAA[i * A + c];
            double lat, rel;
            if (el < 0.0) {  // no edge between the pair: igraph_get_eid fails (shd-topology.c:857)
                nerr++;
                lat = -1.0;
                rel = -1.0;
            } else {
                rel = 1.0;
                rel *= (1.0 - vi);
                rel *= (1.0 - vlossA[c]);
                lat = 0.0;
                lat += el;
                rel *= (1.0 - elossAA[i * A + c]);
                const unsigned long long b = d2bits(lat);
                m = b < m ? b : m;
            }
            const int64_t k = r * (int64_t)A + c;
            out_lr[k] = make_double2(lat, rel);
            out_hops[k] = 1;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long y = __shfl_xor(m, o, 64);
            m = y < m ? y : m;
        }
        if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long x = sm[0];
#pragma unroll
            for (int w = 1; w < 4; w++) x = sm[w] < x ? sm[w] : x;
            if (out_rowmin) out_rowmin[r] = bits2d(x);
            gm = x < gm ? x : gm;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && gm != kInfBits) atomicMin(&stats[ST_GLOBAL_MIN], gm);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nerr += __shfl_xor(nerr, o, 64);
    if ((threadIdx.x & 63) == 0 && nerr) atomicAdd(&stats[ST_ERRORS], (unsigned long long)nerr);
}

// per-row minimum of an installed table (shdtopo_bind_table*: the lazy-runahead bookkeeping)
__global__ void row_min_kernel(int64_t rows, int64_t A, const double2* __restrict__ lr,
                               double* __restrict__ out_rowmin) {
    const int64_t r = blockIdx.x;
    if (r >= rows) return;
    unsigned long long m = kInfBits;
    for (int64_t c = threadIdx.x; c < A; c += blockDim.x) {
        double l = lr[r * A + c].x;
        if (l >= 0.0) { unsigned long long b = d2bits(l); m = b < m ? b : m; }
    }
    __shared__ unsigned long long sm;
    if (threadIdx.x == 0) sm = kInfBits;
    __syncthreads();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long y = __shfl_xor(m, o, 64);
        m = y < m ? y : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMin(&sm, m);
    __syncthreads();
    if (threadIdx.x == 0) out_rowmin[r] = bits2d(sm);
}

// ------------------------------------------------------------------------------------------
// packet route: worker_schedulePacket (shd-worker.c:332-370) + clamp (shd-worker.c:310-324).
// 53 B per packet: 24 B of inputs, one 16-B {lat, rel} record gather, 13 B of outputs.
// Each thread takes kRouteU packets of a 256 x kRouteU tile (coalesced column / state loads) and
// issues all of their record gathers before using any: the gathers are random 16-B reads of a
// table far larger than the caches, so the kernel lives on memory-level parallelism.
// A column outside [0, A) is not routed (delivered 0, time 0, state unchanged) and counted.
// ------------------------------------------------------------------------------------------
#ifndef SHD_ROUTE_U
#define SHD_ROUTE_U 1
#endif
constexpr int kRouteU = SHD_ROUTE_U;  // packets per thread (gathers in flight)

__global__ void __launch_bounds__(256)
packet_route_kernel(int64_t n, const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                    const uint32_t* __restrict__ payload, const uint32_t* __restrict__ state_in,
                    const uint64_t* __restrict__ now, const double2* __restrict__ table, int64_t A,
                    uint64_t jump, int clamp, uint64_t* __restrict__ t_out,
                    uint32_t* __restrict__ state_out, uint8_t* __restrict__ delivered,
                    unsigned long long* __restrict__ bad) {
    const int64_t tile = (int64_t)blockIdx.x * 256 * kRouteU + threadIdx.x;
    int64_t idx[kRouteU];
    bool ok[kRouteU];
#pragma unroll
    for (int j = 0; j < kRouteU; j++) {
        const int64_t k = tile + (int64_t)j * 256;
        int64_t x = -1;
        if (k < n) {
            const uint32_t a = (uint32_t)__builtin_nontemporal_load(src + k);
            const uint32_t b = (uint32_t)__builtin_nontemporal_load(dst + k);
            if ((int64_t)a < A && (int64_t)b < A) x = (int64_t)a * A + b;
        }
        idx[j] = x;
        ok[j] = x >= 0;
    }
    double2 rec[kRouteU];
#pragma unroll
    for (int j = 0; j < kRouteU; j++) rec[j] = ok[j] ? table[idx[j]] : make_double2(0.0, -1.0);
    uint32_t nbad = 0;
#pragma unroll
    for (int j = 0; j < kRouteU; j++) {
        const int64_t k = tile + (int64_t)j * 256;
        if (k >= n) break;
        const uint32_t s0 = __builtin_nontemporal_load(state_in + k);
        const uint32_t pay = __builtin_nontemporal_load(payload + k);
        const uint64_t tnow = __builtin_nontemporal_load(now + k);
        uint64_t t = 0;
        uint8_t dl = 0;
        uint32_t next = s0;
        if (ok[j]) {
            // glibc rand_r: three LCG steps, 11 + 10 + 10 bits
            next = next * 1103515245u + 12345u;
            uint32_t r = (next / 65536u) % 2048u;
            next = next * 1103515245u + 12345u;
            r = (r << 10) ^ ((next / 65536u) % 1024u);
            next = next * 1103515245u + 12345u;
            r = (r << 10) ^ ((next / 65536u) % 1024u);
            const double chance = (double)(int32_t)r / 2147483647.0;
            if (chance <= rec[j].y || pay == 0u) {
                const uint64_t delay = (uint64_t)ceil(rec[j].x * 1000000.0);
                t = tnow + delay;
                if (clamp) {
                    const uint64_t minTime = tnow + jump;
                    if (t < minTime) t = minTime;
                }
                dl = 1;
            }
        } else {
            nbad++;
        }
        __builtin_nontemporal_store(t, t_out + k);
        __builtin_nontemporal_store(next, state_out + k);
        delivered[k] = dl;
    }
    if (nbad && bad) atomicAdd(bad, (unsigned long long)nbad);
}

__global__ void fill_u64_kernel(unsigned long long* p, unsigned long long v, int64_t n) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n;
         k += (int64_t)gridDim.x * blockDim.x)
        p[k] = v;
}

// p[b * stride + i] = v for b < nb, i < n (the same window of every slot's block)
__global__ void fill_u64_strided_kernel(unsigned long long* p, unsigned long long v, int64_t nb,
                                        int64_t stride, int64_t n) {
    const int64_t tot = nb * n;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < tot;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = k / n;
        p[b * stride + (k - b * n)] = v;
    }
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static int grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 256 * 16) g = 256 * 16;  // 16 workgroups per CU, grid-stride beyond
    if (g < 1) g = 1;
    return (int)g;
}

hipError_t launch_pair_table_complete(int A, int64_t row0, int64_t rows, const double* elatAA,
                                      const double* elossAA, const double* vlossA, double2* out_lr,
                                      uint16_t* out_hops, double* out_rowmin,
                                      unsigned long long* d_stats, hipStream_t stream) {
    if (rows <= 0 || A <= 0) return hipSuccess;
    // one workgroup per row (a single launch: records, hops, row minima, global minimum)
    const int64_t g = rows < 256 * 16 ? rows : 256 * 16;
    hipLaunchKernelGGL(pair_table_complete_kernel, dim3((unsigned)g), dim3(256), 0, stream, A,
                       row0, rows, elatAA, elossAA, vlossA, out_lr, out_hops, out_rowmin,
                       d_stats);
    return hipGetLastError();
}

hipError_t launch_packet_route(int64_t n, const int32_t* src, const int32_t* dst,
                               const uint32_t* payload, const uint32_t* state_in,
                               const uint64_t* now, const double2* table, int64_t A,
                               uint64_t jump, int clamp, uint64_t* t_out, uint32_t* state_out,
                               uint8_t* delivered, unsigned long long* d_bad, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const int64_t tiles = (n + 256 * kRouteU - 1) / (256 * kRouteU);
    if (tiles > INT32_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(packet_route_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, n, src,
                       dst, payload, state_in, now, table, A, jump, clamp, t_out, state_out,
                       delivered, d_bad);
    return hipGetLastError();
}

hipError_t launch_row_min(int64_t rows, int64_t A, const double2* lr, double* out_rowmin,
                          hipStream_t stream) {
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(row_min_kernel, dim3((unsigned)rows), dim3(256), 0, stream, rows, A, lr,
                       out_rowmin);
    return hipGetLastError();
}

hipError_t launch_fill_u64(unsigned long long* p, unsigned long long v, int64_t n,
                           hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_u64_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, p, v, n);
    return hipGetLastError();
}

hipError_t launch_fill_u64_strided(unsigned long long* p, unsigned long long v, int64_t nb,
                                   int64_t stride, int64_t n, hipStream_t stream) {
    if (nb <= 0 || n <= 0) return hipSuccess;
    hipLaunchKernelGGL(fill_u64_strided_kernel, dim3(grid_for(nb * n, 256)), dim3(256), 0, stream,
                       p, v, nb, stride, n);
    return hipGetLastError();
}

hipError_t preload_kernels_module() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)packet_route_kernel);
}

}  // namespace shdtopo
