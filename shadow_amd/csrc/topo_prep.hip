// topo_prep.hip -- the once-per-topology graph preparation, on the GPU.
//
// What it builds is the device side of struct _Topology (shd-topology.c:9-53 holds an igraph_t and
// its edge weights; _topology_extractEdgeWeights, :399-432): the relabelled CSR the batch SSSP
// walks, and the landmark data its filter needs.  In the reference this work does not exist (igraph
// walks its own incidence lists inside every Dijkstra, shd-topology.c:762); here it is paid once
// per topology, before the first table, so it is part of the cold build a Shadow run waits for.
// Host work is reduced to copying the parsed edge arrays in and four per-vertex arrays out.
//
// Steps (all on the library's stream; E = edges incl. self loops, 2E' = adjacency entries):
//   1. degrees (self loops excluded) and each vertex's lowest-id self loop (igraph_get_eid's);
//   2. relabel: vertices by degree, descending (stable radix sort), then the tail grouped by its
//      highest-ranked hub neighbour (second stable sort) -- a hub expansion then touches runs of
//      tail distance lines;
//   3. adjacency: every undirected edge as two entries sorted by (row, neighbour, edge id) with
//      one 64-bit-key stable radix sort (rows ascending by neighbour, parallel edges by id);
//   4. pi = d(h0, .) from the top hub h0 = vertex 0: a frontier Bellman-Ford to the unique
//      monotone-rounding fixpoint (every add one IEEE add: the same bits as any Dijkstra);
//   5. the h0 tree: parent(v) = argmin (d(u), u) over the tight edges (u, v) with d(u) < d(v) --
//      the tree a binary-heap Dijkstra from h0 keyed (d, vertex) produces;
//   6. kappa0(v) = min over v's row of w - pi(col), the records' {f16 pi up, f16 kappa0 down}
//      field, pi max;
//   7. the kappa-sorted relaxation copy: rows sorted by f32(w - pi(col)) rounded down (one global
//      radix sort on (row, key)), the h0-tree edge flagged, kappa probes and kappa0.
// Row-parallel steps take a wavefront per segment of a hub row (ids < hs.rows, the long rows after
// step 2; at most kHubSeg entries per segment, HubSegs) and a thread per tail row.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "topo_dev_common.h"

namespace shdtopo {

namespace {

using namespace dev;

#define PCHK(expr)                          \
    do {                                    \
        const hipError_t e_ = (expr);       \
        if (e_ != hipSuccess) return e_;    \
    } while (0)

template <class T>
struct Tmp {  // scratch device buffer, freed on scope exit
    T* p = nullptr;
    ~Tmp() {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc((void**)&p, sizeof(T) * (n ? n : 1)); }
};

constexpr int kPB = 256;  // threads per block of the prep kernels

unsigned grid_for(int64_t n) {
    const int64_t g = (n + kPB - 1) / kPB;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 64));
}

__device__ __forceinline__ int64_t gtid() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ int64_t gstride() { return (int64_t)gridDim.x * blockDim.x; }

// --- directed roundings of the record fields (bounds never tighten) ---
// largest f16 <= x (-inf if none; NaN -> -inf), smallest f16 >= x (+inf if none; NaN -> +inf)
__device__ __forceinline__ uint32_t f16_dn(double x) {
    if (isnan(x)) return 0xFC00u;
    uint32_t b = (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)(float)x);
    if ((double)(float)__builtin_bit_cast(_Float16, (unsigned short)b) > x) {
        if ((b & 0x7FFFu) == 0u) b = 0x8001u;
        else if (b & 0x8000u) b++;
        else b--;
    }
    return b == 0x7C00u ? 0x7BFFu : (b & 0xFFFFu);  // +inf input: the largest finite half
}
__device__ __forceinline__ uint32_t f16_up(double x) {
    if (isnan(x)) return 0x7C00u;
    uint32_t b = (uint32_t)__builtin_bit_cast(unsigned short, (_Float16)(float)x);
    if ((double)(float)__builtin_bit_cast(_Float16, (unsigned short)b) < x) {
        if ((b & 0x7FFFu) == 0u) b = 0x0001u;
        else if (b & 0x8000u) b--;
        else b++;
    }
    return b == 0xFC00u ? 0xFBFFu : (b & 0xFFFFu);  // -inf input: the smallest finite half
}
__device__ __forceinline__ float f32_dn(double x) {
    if (isnan(x)) return -INFINITY;
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}
__device__ __forceinline__ float f32_up(double x) {
    if (isnan(x)) return INFINITY;
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}
// f32 bits -> u32 that orders like the value
__device__ __forceinline__ uint32_t f32_order(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ double rec_w(const uint32_t* adj, uint32_t k) {
    return __hiloint2double((int)adj[kAdjWords * k + 3], (int)adj[kAdjWords * k + 2]);
}

// ---------------------------------------------------------------------------------------------
// 1. degrees + lowest-id self loop
// ---------------------------------------------------------------------------------------------
__global__ void prep_degree_kernel(int64_t E, const int32_t* __restrict__ eu,
                                   const int32_t* __restrict__ ev, uint32_t* __restrict__ deg,
                                   uint32_t* __restrict__ selfE,
                                   unsigned long long* __restrict__ nadj) {
    unsigned long long n = 0;
    for (int64_t e = gtid(); e < E; e += gstride()) {
        const int32_t a = eu[e], b = ev[e];
        if (a == b) {
            atomicMin(&selfE[a], (uint32_t)e);
        } else {
            atomicAdd(&deg[a], 1u);
            atomicAdd(&deg[b], 1u);
            n += 2;
        }
    }
    n = wave_sum_u64(n);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(nadj, n);
}

// ---------------------------------------------------------------------------------------------
// 2. relabel
// ---------------------------------------------------------------------------------------------
__global__ void prep_degkey_kernel(int64_t V, const uint32_t* __restrict__ deg,
                                   uint32_t* __restrict__ key, uint32_t* __restrict__ iota) {
    for (int64_t v = gtid(); v < V; v += gstride()) {
        key[v] = 0xFFFFFFFFu - deg[v];  // ascending key = descending degree
        iota[v] = (uint32_t)v;
    }
}

__global__ void prep_hubrank_kernel(int64_t V, uint32_t H, const uint32_t* __restrict__ perm,
                                    int32_t* __restrict__ hubrank, int32_t* __restrict__ primary) {
    for (int64_t i = gtid(); i < V; i += gstride()) {
        hubrank[perm[i]] = i < (int64_t)H ? (int32_t)i : INT32_MAX;
        primary[i] = INT32_MAX;
    }
}

__global__ void prep_primary_kernel(int64_t E, const int32_t* __restrict__ eu,
                                    const int32_t* __restrict__ ev,
                                    const int32_t* __restrict__ hubrank,
                                    int32_t* __restrict__ primary) {
    for (int64_t e = gtid(); e < E; e += gstride()) {
        const int32_t a = eu[e], b = ev[e];
        if (a == b) continue;
        const int32_t rb = hubrank[b], ra = hubrank[a];
        if (rb != INT32_MAX) atomicMin(&primary[a], rb);
        if (ra != INT32_MAX) atomicMin(&primary[b], ra);
    }
}

__global__ void prep_tailkey_kernel(int64_t n, const uint32_t* __restrict__ tail,
                                    const int32_t* __restrict__ primary,
                                    uint32_t* __restrict__ key) {
    for (int64_t i = gtid(); i < n; i += gstride()) key[i] = (uint32_t)primary[tail[i]];
}

__global__ void prep_relabel_kernel(int64_t V, const uint32_t* __restrict__ perm,
                                    const uint32_t* __restrict__ deg,
                                    const uint32_t* __restrict__ selfE,
                                    const double* __restrict__ elat,
                                    const double* __restrict__ eloss,
                                    const double* __restrict__ vloss_in,
                                    uint32_t* __restrict__ inv, uint32_t* __restrict__ degn,
                                    double* __restrict__ vloss, double* __restrict__ selfLat,
                                    double* __restrict__ selfLoss) {
    for (int64_t i = gtid(); i < V; i += gstride()) {
        const uint32_t o = perm[i];
        inv[o] = (uint32_t)i;
        degn[i] = deg[o];
        vloss[i] = vloss_in[o];
        const uint32_t s = selfE[o];
        selfLat[i] = s == 0xFFFFFFFFu ? (double)NAN : elat[s];
        selfLoss[i] = s == 0xFFFFFFFFu ? 0.0 : eloss[s];
    }
    if (gtid() == 0) degn[V] = 0u;  // the exclusive scan's extra element: rowptr[V] = 2E'
}

// ---------------------------------------------------------------------------------------------
// 3. adjacency entries
// ---------------------------------------------------------------------------------------------
__global__ void prep_entry_kernel(int64_t E, int64_t V, const int32_t* __restrict__ eu,
                                  const int32_t* __restrict__ ev, const uint32_t* __restrict__ inv,
                                  unsigned long long* __restrict__ key,
                                  uint32_t* __restrict__ val, int mode) {
    const unsigned long long sentinel = (unsigned long long)V << 32;  // self loops sort last
    for (int64_t e = gtid(); e < E; e += gstride()) {
        const int32_t a = eu[e], b = ev[e];
        unsigned long long k0 = sentinel, k1 = sentinel;
        if (a != b) {
            const unsigned long long na = inv[a], nb = inv[b];
            k0 = (na << 32) | nb;  // a's row (out-entry of a directed edge a -> b)
            k1 = (nb << 32) | na;  // b's row (in-entry)
        }
        if (mode == kAdjBoth) {
            key[2 * e] = k0;
            key[2 * e + 1] = k1;
            val[2 * e] = val[2 * e + 1] = (uint32_t)e;
        } else {
            key[e] = mode == kAdjOut ? k0 : k1;
            val[e] = (uint32_t)e;
        }
    }
}

// rowptr[v] = the first sorted entry of row >= v (rows 0..V; self loops sort as row V)
__global__ void prep_rowptr_kernel(int64_t V, int64_t n, const unsigned long long* __restrict__ key,
                                   uint32_t* __restrict__ rowptr) {
    for (int64_t v = gtid(); v <= V; v += gstride()) {
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if ((int64_t)(key[mid] >> 32) < v) lo = mid + 1; else hi = mid;
        }
        rowptr[v] = (uint32_t)lo;
    }
}

__global__ void prep_fill_adj_kernel(int64_t nadj, const unsigned long long* __restrict__ key,
                                     const uint32_t* __restrict__ eid,
                                     const double* __restrict__ elat,
                                     const double* __restrict__ eloss, uint32_t* __restrict__ adj,
                                     double* __restrict__ aloss) {
    for (int64_t k = gtid(); k < nadj; k += gstride()) {
        const uint32_t e = eid[k];
        const unsigned long long wb = d2bits(elat[e]);
        uint4 r;
        r.x = (uint32_t)key[k];
        r.y = 0u;
        r.z = (uint32_t)wb;
        r.w = (uint32_t)(wb >> 32);
        reinterpret_cast<uint4*>(adj)[k] = r;
        if (aloss) aloss[k] = eloss[e];
    }
}

// ---------------------------------------------------------------------------------------------
// 4. pi = d(h0, .): frontier Bellman-Ford (label-correcting; the fixpoint is unique)
// ---------------------------------------------------------------------------------------------
__global__ void h0_fdeg_kernel(uint32_t nF, const uint32_t* __restrict__ F,
                               const uint32_t* __restrict__ rowptr, uint32_t* __restrict__ fdeg) {
    for (int64_t i = gtid(); i <= (int64_t)nF; i += gstride())
        fdeg[i] = i < (int64_t)nF ? rowptr[F[i] + 1] - rowptr[F[i]] : 0u;
}

constexpr uint32_t kEPB = 2048;  // frontier edges per block step

__global__ void __launch_bounds__(kPB)
h0_relax_kernel(uint32_t nF, const uint32_t* __restrict__ F, const uint32_t* __restrict__ foff,
                const uint32_t* __restrict__ rowptr, const uint32_t* __restrict__ adj,
                unsigned long long* __restrict__ d, uint32_t* __restrict__ inq, uint32_t stamp,
                uint32_t* __restrict__ N, uint32_t* __restrict__ nN) {
    __shared__ uint32_t soff[kEPB + 1];
    __shared__ uint32_t s_i0, s_n;
    const uint32_t total = foff[nF];
    const uint32_t tid = threadIdx.x;
    for (uint32_t e0 = blockIdx.x * kEPB; e0 < total; e0 += gridDim.x * kEPB) {
        const uint32_t e1 = min(e0 + kEPB, total);
        if (tid == 0) {
            // frontier slots [i0, i1] hold edges [e0, e1): last slot with foff <= e, by search
            uint32_t lo = 0, hi = nF - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (foff[mid] <= e0) lo = mid; else hi = mid - 1;
            }
            const uint32_t i0 = lo;
            hi = nF - 1;
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (foff[mid] <= e1 - 1) lo = mid; else hi = mid - 1;
            }
            s_i0 = i0;
            s_n = lo - i0 + 1;  // <= kEPB: every frontier vertex has an edge
        }
        __syncthreads();
        const uint32_t i0 = s_i0, n = min(s_n, kEPB + 1);
        for (uint32_t j = tid; j < n; j += kPB) soff[j] = foff[i0 + j];
        __syncthreads();
        for (uint32_t eb = e0; eb < e1; eb += kPB) {  // uniform trip count: the ballot below
            const uint32_t e = eb + tid;
            bool push = false;
            uint32_t v = 0;
            if (e < e1) {
                uint32_t lo = 0, hi = n - 1;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1) >> 1;
                    if (soff[mid] <= e) lo = mid; else hi = mid - 1;
                }
                const uint32_t u = F[i0 + lo];
                const uint32_t k = rowptr[u] + (e - soff[lo]);
                v = adj[kAdjWords * k];
                const double nd = __dadd_rn(bits2d(ld_l2_u64(&d[u])), rec_w(adj, k));
                const unsigned long long nb = d2bits(nd);
                if (nb < ld_l2_u64(&d[v])) {
                    const unsigned long long old = atomicMin(&d[v], nb);
                    if (nb < old) push = atomicExch(&inq[v], stamp) != stamp;
                }
            }
            const unsigned long long m = __ballot(push);
            if (m) {
                const int lane = threadIdx.x & 63;
                const int leader = __ffsll((long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(nN, (uint32_t)__popcll(m));
                base = __shfl(base, leader, 64);
                if (push) N[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = v;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// 5. + 6. the h0 tree, kappa0, pi max (a wavefront per hub row, a thread per tail row)
// ---------------------------------------------------------------------------------------------
struct TreeBest {
    unsigned long long du;
    uint32_t u, k;
};
__device__ __forceinline__ bool tb_less(const TreeBest& a, const TreeBest& b) {
    return a.du < b.du || (a.du == b.du && a.u < b.u);
}

__device__ __forceinline__ void tree_scan(const uint32_t* adj, const double* pot, uint32_t v,
                                          double dv, uint32_t b, uint32_t e, uint32_t step,
                                          TreeBest& best, double& kmin) {
    for (uint32_t k = b; k < e; k += step) {
        const uint32_t u = adj[kAdjWords * k];
        const double w = rec_w(adj, k);
        const double du = pot[u];
        const double kap = isfinite(du) ? w - du : -INFINITY;
        kmin = kap < kmin ? kap : kmin;
        if (u != v && du < dv && __dadd_rn(du, w) == dv) {
            const TreeBest c{d2bits(du), u, k};
            if (tb_less(c, best)) best = c;
        }
    }
}

__device__ __forceinline__ void tree_store(uint32_t v, const TreeBest& best, const uint32_t* adj,
                                           const double* aloss, uint32_t* sptPar, uint32_t* spt,
                                           double kmin, double* kap0d, int what) {
    if (what & kTreeKappa) kap0d[v] = kmin;
    if (!(what & kTreeParents)) return;
    const bool ok = best.u != 0xFFFFFFFFu;
    sptPar[v] = ok ? best.u : 0xFFFFFFFFu;
    // 32-B record {parent, slot, f64 w, f64 loss, pad}: a walk hop reads it as one line
    const unsigned long long lb = ok ? d2bits(aloss[best.k]) : 0ull;
    uint4 r = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    if (ok) r = make_uint4(best.u, best.k, adj[kAdjWords * best.k + 2], adj[kAdjWords * best.k + 3]);
    reinterpret_cast<uint4*>(spt)[2 * (size_t)v] = r;
    reinterpret_cast<uint4*>(spt)[2 * (size_t)v + 1] = make_uint4((uint32_t)lb, (uint32_t)(lb >> 32), 0u, 0u);
}

__device__ __forceinline__ void tb_wave_min(TreeBest& best, double& kmin) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        TreeBest y;
        y.du = __shfl_xor(best.du, o, 64);
        y.u = __shfl_xor(best.u, o, 64);
        y.k = __shfl_xor(best.k, o, 64);
        if (tb_less(y, best)) best = y;
        const double km = __shfl_xor(kmin, o, 64);
        kmin = km < kmin ? km : kmin;
    }
}

__global__ void __launch_bounds__(kPB)
prep_tree_kernel(int64_t V, HubSegs hs, const uint32_t* __restrict__ rowptr,
                 const uint32_t* __restrict__ adj, const double* __restrict__ aloss,
                 const double* __restrict__ pot, uint32_t* __restrict__ sptPar,
                 uint32_t* __restrict__ spt, double* __restrict__ kap0d, unsigned long long* __restrict__ pimax,
                 TreeBest* __restrict__ pbest, double* __restrict__ pkmin, int what) {
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t nw = gstride() >> 6;
    const TreeBest none{~0ull, 0xFFFFFFFFu, 0xFFFFFFFFu};
    // hub rows: a wavefront per segment; a row cut in several leaves partials (prep_tree_multi)
    for (int64_t s = gtid() >> 6; s < (int64_t)hs.nseg; s += nw) {
        const uint2 sg = hs.seg[s];
        const uint32_t v = sg.x, r0 = rowptr[v], r1 = rowptr[v + 1];
        const uint32_t e = min(sg.y + kHubSeg, r1);
        TreeBest best = none;
        double kmin = INFINITY;
        const double dv = pot[v];
        tree_scan(adj, pot, v, v == 0 ? -INFINITY : dv, sg.y + lane, e, 64u, best, kmin);
        tb_wave_min(best, kmin);
        if (lane == 0) {
            if (sg.y == r0 && e == r1) {
                tree_store(v, best, adj, aloss, sptPar, spt, kmin, kap0d, what);
            } else {
                pbest[s] = best;
                pkmin[s] = kmin;
            }
        }
    }
    // tail rows: a thread each
    unsigned long long pm = 0;
    for (int64_t v = gtid(); v < V; v += gstride()) {
        const double dv = pot[v];
        if (isfinite(dv)) pm = d2bits(dv) > pm ? d2bits(dv) : pm;
        if (v < (int64_t)hs.rows) continue;
        TreeBest best = none;
        double kmin = INFINITY;
        tree_scan(adj, pot, (uint32_t)v, dv, rowptr[v], rowptr[v + 1], 1u, best, kmin);
        tree_store((uint32_t)v, best, adj, aloss, sptPar, spt, kmin, kap0d, what);
    }
    pm = wave_min_u64(~pm);
    if (lane == 0 && pm != ~0ull) atomicMax(pimax, ~pm);
}

// the rows cut in several segments: a wavefront each combines its segments' partials
__global__ void __launch_bounds__(kPB)
prep_tree_multi_kernel(HubSegs hs, const uint32_t* __restrict__ adj,
                       const double* __restrict__ aloss, uint32_t* __restrict__ sptPar,
                       uint32_t* __restrict__ spt, double* __restrict__ kap0d, const TreeBest* __restrict__ pbest,
                       const double* __restrict__ pkmin, int what) {
    const uint32_t lane = threadIdx.x & 63u;
    for (int64_t m = gtid() >> 6; m < (int64_t)hs.nmulti; m += gstride() >> 6) {
        const uint4 mr = hs.multi[m];
        TreeBest best{~0ull, 0xFFFFFFFFu, 0xFFFFFFFFu};
        double kmin = INFINITY;
        for (uint32_t i = lane; i < mr.z; i += 64u) {
            const TreeBest c = pbest[mr.y + i];
            if (tb_less(c, best)) best = c;
            const double km = pkmin[mr.y + i];
            kmin = km < kmin ? km : kmin;
        }
        tb_wave_min(best, kmin);
        if (lane == 0) tree_store(mr.x, best, adj, aloss, sptPar, spt, kmin, kap0d, what);
    }
}

// the records' 32-bit field: {f16 pi(col) rounded up, f16 kappa0(col) rounded down} (or the f32 pi
// rounded up when the record does not carry kappa0)
__global__ void prep_recfield_kernel(int64_t nadj, uint32_t* __restrict__ adj,
                                     const double* __restrict__ pot,
                                     const double* __restrict__ kap0d) {
    for (int64_t k = gtid(); k < nadj; k += gstride()) {
        const uint32_t c = adj[kAdjWords * k];
        const double pv = pot[c];
        uint32_t pb;
        if (kKapInRec) pb = (f16_up(isfinite(pv) ? pv : INFINITY) << 16) | f16_dn(kap0d[c]);
        else pb = __float_as_uint(isfinite(pv) ? f32_up(pv) : INFINITY);
        adj[kAdjWords * k + 1] = pb;
    }
}

// ---------------------------------------------------------------------------------------------
// 7. kappa-sorted relaxation copy
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kPB)
kap_key_kernel(int64_t V, HubSegs hs, const uint32_t* __restrict__ rowptr,
               const uint32_t* __restrict__ adj, const double* __restrict__ pot,
               unsigned long long* __restrict__ key, uint32_t* __restrict__ idx) {
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t nw = gstride() >> 6;
    auto one = [&](uint32_t v, uint32_t k) {
        const double pv = pot[adj[kAdjWords * k]];
        const double kd = isfinite(pv) ? rec_w(adj, k) - pv : -INFINITY;
        key[k] = ((unsigned long long)v << 32) | f32_order(f32_dn(kd));
        idx[k] = k;
    };
    for (int64_t s = gtid() >> 6; s < (int64_t)hs.nseg; s += nw) {
        const uint2 sg = hs.seg[s];
        const uint32_t e = min(sg.y + kHubSeg, rowptr[sg.x + 1]);
        for (uint32_t k = sg.y + lane; k < e; k += 64u) one(sg.x, k);
    }
    for (int64_t v = (int64_t)hs.rows + gtid(); v < V; v += gstride())
        for (uint32_t k = rowptr[v]; k < rowptr[v + 1]; k++) one((uint32_t)v, k);
}

__global__ void kap_gather_kernel(int64_t nadj, const unsigned long long* __restrict__ key,
                                  const uint32_t* __restrict__ idx,
                                  const uint32_t* __restrict__ adj,
                                  const uint32_t* __restrict__ sptPar,
                                  uint32_t* __restrict__ adjk, float* __restrict__ kap) {
    for (int64_t i = gtid(); i < nadj; i += gstride()) {
        const unsigned long long kk = key[i];
        const uint32_t row = (uint32_t)(kk >> 32), o = (uint32_t)kk;
        uint4 r = reinterpret_cast<const uint4*>(adj)[idx[i]];
        // bit 31 of the relaxation copy's column: the h0-tree edge into the column
        if (sptPar[r.x] == row) r.x |= 0x80000000u;
        reinterpret_cast<uint4*>(adjk)[i] = r;
        kap[i] = __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
    }
}

__global__ void kap_probe_kernel(int64_t V, const uint32_t* __restrict__ rowptr,
                                 const float* __restrict__ kap, float* __restrict__ ksum,
                                 float* __restrict__ kap0) {
    for (int64_t v = gtid(); v < V; v += gstride()) {
        const uint32_t b = rowptr[v], n = rowptr[v + 1] - b;
#pragma unroll
        for (int q = 0; q < kKProbes; q++) {
            const uint32_t pq = (1u << q) - 1u;  // 0, 1, 3, 7, 15, 31, 63, 127
            ksum[(size_t)kKProbes * v + q] = pq < n ? kap[b + pq] : INFINITY;
        }
        kap0[v] = n ? kap[b] : INFINITY;
    }
}

// ---------------------------------------------------------------------------------------------
// the heap replay's incidence CSR (ReplayCSR, topo_device.h): igraph_incident order
// ---------------------------------------------------------------------------------------------
// entries (x, y, e) of every non-loop edge (both directions when undirected), keyed by
// (relabelled x, ORIGINAL y): a stable sort gives igraph's order in each row -- ascending original
// neighbour, a parallel group by ascending edge id
__global__ void rp_entry_kernel(int64_t E, int directed, const int32_t* __restrict__ eu,
                                const int32_t* __restrict__ ev, const uint32_t* __restrict__ inv,
                                unsigned long long* __restrict__ key, uint32_t* __restrict__ val,
                                unsigned long long sentinel) {
    for (int64_t e = gtid(); e < E; e += gstride()) {
        const int32_t a = eu[e], b = ev[e];
        unsigned long long k0 = sentinel, k1 = sentinel;
        if (a != b) {
            k0 = ((unsigned long long)inv[a] << 32) | (uint32_t)b;
            if (!directed) k1 = ((unsigned long long)inv[b] << 32) | (uint32_t)a;
        }
        if (directed) {
            key[e] = k0;
            val[e] = (uint32_t)e;
        } else {
            key[2 * e] = k0;
            key[2 * e + 1] = k1;
            val[2 * e] = val[2 * e + 1] = (uint32_t)e;
        }
    }
}

// group starts (a parallel group merges into one entry) and the entries per row
__global__ void rp_group_kernel(int64_t n, const unsigned long long* __restrict__ key,
                                unsigned long long sentinel, uint32_t* __restrict__ start,
                                uint32_t* __restrict__ rowcnt) {
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const unsigned long long k = key[i];
        const bool s = k != sentinel && (i == 0 || key[i - 1] != k);
        start[i] = s ? 1u : 0u;
        if (s) atomicAdd(&rowcnt[k >> 32], 1u);
    }
}

__global__ void rp_fill_kernel(int64_t n, const unsigned long long* __restrict__ key,
                               const uint32_t* __restrict__ eid, const uint32_t* __restrict__ start,
                               const uint32_t* __restrict__ gpos, int directed,
                               const uint32_t* __restrict__ inv, const double* __restrict__ pot,
                               const double* __restrict__ elat, const double* __restrict__ eloss,
                               uint4* __restrict__ rec, uint32_t* __restrict__ own,
                               double2* __restrict__ hop) {
    for (int64_t i = gtid(); i < n; i += gstride()) {
        if (!start[i]) continue;
        const unsigned long long k = key[i];
        const uint32_t e0 = eid[i];  // the group's lowest edge id: igraph_get_eid's edge
        double w = elat[e0];
        for (int64_t j = i + 1; j < n && key[j] == k; j++) w = fmin(w, elat[eid[j]]);
        const uint32_t g = gpos[i];
        const uint32_t y = inv[(uint32_t)k];
        // pi(y) = d(h0, y) rounded up to f32: the replay's landmark skip (topo_replay.hip)
        float pf = INFINITY;
        if (pot) {  // directed: pi = d(h0 -> y) over the out-rows, the same bound
            const double p = pot[y];
            if (isfinite(p)) pf = f32_up(p);
        }
        const unsigned long long wb = d2bits(w);
        rec[g] = make_uint4(y, __float_as_uint(pf), (uint32_t)wb, (uint32_t)(wb >> 32));
        own[g] = (uint32_t)(k >> 32);
        hop[g] = make_double2(elat[e0], eloss[e0]);
    }
}

__global__ void prep_fill_u64_kernel(unsigned long long* __restrict__ p, unsigned long long v,
                                     int64_t n) {
    for (int64_t i = gtid(); i < n; i += gstride()) p[i] = v;
}

int bitlen(uint64_t x) {
    int b = 0;
    while (x) { b++; x >>= 1; }
    return b;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// launchers (topo_device.h)
// ---------------------------------------------------------------------------------------------
hipError_t prep_degrees(int64_t V, int64_t E, const int32_t* eu, const int32_t* ev, uint32_t* deg,
                        uint32_t* selfE, int64_t* nadj, hipStream_t st) {
    Tmp<unsigned long long> n;
    PCHK(n.alloc(1));
    PCHK(hipMemsetAsync(deg, 0, sizeof(uint32_t) * (size_t)V, st));
    PCHK(hipMemsetAsync(selfE, 0xFF, sizeof(uint32_t) * (size_t)V, st));
    PCHK(hipMemsetAsync(n.p, 0, 8, st));
    if (E > 0)
        hipLaunchKernelGGL(prep_degree_kernel, dim3(grid_for(E)), dim3(kPB), 0, st, E, eu, ev, deg,
                           selfE, n.p);
    PCHK(hipGetLastError());
    unsigned long long h = 0;
    PCHK(hipMemcpyAsync(&h, n.p, 8, hipMemcpyDeviceToHost, st));
    PCHK(hipStreamSynchronize(st));
    *nadj = (int64_t)h;
    return hipSuccess;
}

hipError_t prep_relabel(int64_t V, int64_t E, uint32_t H, const int32_t* eu, const int32_t* ev,
                        const uint32_t* deg, const uint32_t* selfE, const double* elat,
                        const double* eloss, const double* vloss_in, uint32_t* perm,
                        uint32_t* inv, uint32_t* rowptr, double* vloss, double* selfLat,
                        double* selfLoss, hipStream_t st) {
    Tmp<uint32_t> key, key2, iota, degn, tkey, tval;
    Tmp<int32_t> hubrank, primary;
    Tmp<unsigned char> tmp;
    PCHK(key.alloc(V));
    PCHK(key2.alloc(V));
    PCHK(iota.alloc(V));
    PCHK(degn.alloc(V + 1));
    const unsigned gv = grid_for(V);
    hipLaunchKernelGGL(prep_degkey_kernel, dim3(gv), dim3(kPB), 0, st, V, deg, key.p, iota.p);
    PCHK(hipGetLastError());
    size_t tb = 0, tb2 = 0, tb3 = 0;
    PCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key.p, key2.p, iota.p, perm, (int)V, 0, 32,
                                            st));
    PCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, degn.p, rowptr, (int)(V + 1), st));
    if (H < V)
        PCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb3, key.p, key2.p, iota.p, perm,
                                                (int)(V - H), 0, 32, st));
    PCHK(tmp.alloc(std::max(tb, std::max(tb2, tb3))));
    PCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, key.p, key2.p, iota.p, perm, (int)V, 0, 32,
                                            st));
    if (H < V) {
        // the tail grouped by its highest-ranked hub neighbour ("primary hub"), stable
        PCHK(hubrank.alloc(V));
        PCHK(primary.alloc(V));
        PCHK(tkey.alloc(V - H));
        PCHK(tval.alloc(V - H));
        hipLaunchKernelGGL(prep_hubrank_kernel, dim3(gv), dim3(kPB), 0, st, V, H, perm, hubrank.p,
                           primary.p);
        PCHK(hipGetLastError());
        hipLaunchKernelGGL(prep_primary_kernel, dim3(grid_for(E)), dim3(kPB), 0, st, E, eu, ev,
                           hubrank.p, primary.p);
        PCHK(hipGetLastError());
        hipLaunchKernelGGL(prep_tailkey_kernel, dim3(grid_for(V - H)), dim3(kPB), 0, st, V - H,
                           perm + H, primary.p, tkey.p);
        PCHK(hipGetLastError());
        PCHK(hipMemcpyAsync(tval.p, perm + H, sizeof(uint32_t) * (size_t)(V - H),
                            hipMemcpyDeviceToDevice, st));
        PCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb3, tkey.p, key2.p, tval.p, perm + H,
                                                (int)(V - H), 0, 32, st));
    }
    hipLaunchKernelGGL(prep_relabel_kernel, dim3(gv), dim3(kPB), 0, st, V, perm, deg, selfE, elat,
                       eloss, vloss_in, inv, degn.p, vloss, selfLat, selfLoss);
    PCHK(hipGetLastError());
    PCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb2, degn.p, rowptr, (int)(V + 1), st));
    return hipStreamSynchronize(st);  // the scratch is freed on return
}

hipError_t prep_adjacency(int64_t V, int64_t E, int64_t nadj, const int32_t* eu, const int32_t* ev,
                          const uint32_t* inv, const double* elat, const double* eloss,
                          uint32_t* adj, double* aloss, hipStream_t st, int mode,
                          uint32_t* rowptr) {
    const int64_t n = mode == kAdjBoth ? 2 * E : E;  // entries incl. the self loops' sentinels
    if (nadj <= 0 && !(mode != kAdjBoth && rowptr)) return hipSuccess;
    Tmp<unsigned long long> k0, k1;
    Tmp<uint32_t> v0, v1;
    Tmp<unsigned char> tmp;
    PCHK(k0.alloc(std::max<int64_t>(1, n)));
    PCHK(k1.alloc(std::max<int64_t>(1, n)));
    PCHK(v0.alloc(std::max<int64_t>(1, n)));
    PCHK(v1.alloc(std::max<int64_t>(1, n)));
    if (E > 0) {
        hipLaunchKernelGGL(prep_entry_kernel, dim3(grid_for(E)), dim3(kPB), 0, st, E, V, eu, ev,
                           inv, k0.p, v0.p, mode);
        PCHK(hipGetLastError());
        const int endbit = 32 + bitlen((uint64_t)V);
        size_t tb = 0;
        PCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0.p, k1.p, v0.p, v1.p, (int)n, 0,
                                                endbit, st));
        PCHK(tmp.alloc(tb));
        PCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k0.p, k1.p, v0.p, v1.p, (int)n, 0,
                                                endbit, st));
    }
    if (nadj > 0) {
        hipLaunchKernelGGL(prep_fill_adj_kernel, dim3(grid_for(nadj)), dim3(kPB), 0, st, nadj,
                           k1.p, v1.p, elat, eloss, adj, aloss);
        PCHK(hipGetLastError());
    }
    if (mode != kAdjBoth && rowptr) {
        hipLaunchKernelGGL(prep_rowptr_kernel, dim3(grid_for(V + 1)), dim3(kPB), 0, st, V,
                           E > 0 ? n : 0, k1.p, rowptr);
        PCHK(hipGetLastError());
    }
    return hipStreamSynchronize(st);
}

hipError_t prep_h0_distances(int64_t V, const uint32_t* rowptr, const uint32_t* adj, double* pot,
                             int* iterations, hipStream_t st) {
    Tmp<uint32_t> F, N, inq, fdeg, foff, cnt;
    Tmp<unsigned char> tmp;
    PCHK(F.alloc(V));
    PCHK(N.alloc(V));
    PCHK(inq.alloc(V));
    PCHK(fdeg.alloc(V + 1));
    PCHK(foff.alloc(V + 1));
    PCHK(cnt.alloc(1));
    size_t tb = 0;
    PCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, fdeg.p, foff.p, (int)(V + 1), st));
    PCHK(tmp.alloc(tb));
    unsigned long long* d = reinterpret_cast<unsigned long long*>(pot);
    hipLaunchKernelGGL(prep_fill_u64_kernel, dim3(grid_for(V)), dim3(kPB), 0, st, d, kInfBits, V);
    PCHK(hipGetLastError());
    PCHK(hipMemsetAsync(d, 0, 8, st));  // pi(h0) = 0
    PCHK(hipMemsetAsync(inq.p, 0, sizeof(uint32_t) * (size_t)V, st));
    PCHK(hipMemsetAsync(F.p, 0, 4, st));  // frontier = {h0}
    uint32_t nF = V > 0 ? 1u : 0u;
    int it = 0;
    uint32_t* f = F.p;
    uint32_t* n = N.p;
    while (nF > 0) {
        hipLaunchKernelGGL(h0_fdeg_kernel, dim3(grid_for(nF + 1)), dim3(kPB), 0, st, nF, f, rowptr,
                           fdeg.p);
        PCHK(hipGetLastError());
        PCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, fdeg.p, foff.p, (int)(nF + 1), st));
        PCHK(hipMemsetAsync(cnt.p, 0, 4, st));
        hipLaunchKernelGGL(h0_relax_kernel, dim3(1024), dim3(kPB), 0, st, nF, f, foff.p, rowptr,
                           adj, d, inq.p, (uint32_t)(it + 1), n, cnt.p);
        PCHK(hipGetLastError());
        PCHK(hipMemcpyAsync(&nF, cnt.p, 4, hipMemcpyDeviceToHost, st));
        PCHK(hipStreamSynchronize(st));
        std::swap(f, n);
        if (++it > (1 << 24)) return hipErrorUnknown;  // cannot happen: a fixpoint is reached
    }
    *iterations = it;
    return hipSuccess;
}

void hub_segments(const uint32_t* rowptr_head, uint32_t rows, std::vector<uint2>& seg,
                  std::vector<uint4>& multi) {
    seg.clear();
    multi.clear();
    for (uint32_t v = 0; v < rows; v++) {
        const uint32_t r0 = rowptr_head[v], r1 = rowptr_head[v + 1];
        const uint32_t first = (uint32_t)seg.size();
        uint32_t b = r0;
        do {
            seg.push_back(make_uint2(v, b));
            b += kHubSeg;
        } while (b < r1);
        const uint32_t n = (uint32_t)seg.size() - first;
        if (n > 1) multi.push_back(make_uint4(v, first, n, 0u));
    }
}

hipError_t prep_tree(int64_t V, int64_t nadj, const HubSegs& hs, const uint32_t* rowptr,
                     uint32_t* adj, const double* aloss, const double* pot, uint32_t* sptPar,
                     uint32_t* spt, double* piMax, hipStream_t st, int what) {
    Tmp<double> kap0d, pkmin;
    Tmp<unsigned long long> pm;
    Tmp<TreeBest> pbest;
    PCHK(kap0d.alloc(V));
    PCHK(pm.alloc(1));
    PCHK(pbest.alloc(std::max<uint32_t>(1, hs.nseg)));
    PCHK(pkmin.alloc(std::max<uint32_t>(1, hs.nseg)));
    PCHK(hipMemsetAsync(pm.p, 0, 8, st));
    const unsigned g = std::max(grid_for(V), (unsigned)std::min<int64_t>((hs.nseg + 3) / 4, 256 * 64));
    hipLaunchKernelGGL(prep_tree_kernel, dim3(g), dim3(kPB), 0, st, V, hs, rowptr, adj, aloss,
                       pot, sptPar, spt, kap0d.p, pm.p, pbest.p, pkmin.p, what);
    PCHK(hipGetLastError());
    if (hs.nmulti > 0) {
        hipLaunchKernelGGL(prep_tree_multi_kernel, dim3((hs.nmulti + 3) / 4), dim3(kPB), 0, st, hs,
                           adj, aloss, sptPar, spt, kap0d.p, pbest.p, pkmin.p, what);
        PCHK(hipGetLastError());
    }
    if (nadj > 0 && (what & kTreeKappa))
        hipLaunchKernelGGL(prep_recfield_kernel, dim3(grid_for(nadj)), dim3(kPB), 0, st, nadj, adj,
                           pot, kap0d.p);
    PCHK(hipGetLastError());
    unsigned long long h = 0;
    PCHK(hipMemcpyAsync(&h, pm.p, 8, hipMemcpyDeviceToHost, st));
    PCHK(hipStreamSynchronize(st));
    double x;
    memcpy(&x, &h, 8);
    *piMax = x;
    return hipSuccess;
}

hipError_t launch_kappa_copy(int64_t V, int64_t nadj, const HubSegs& hs, const uint32_t* rowptr,
                             const uint32_t* adj, const double* pot, const uint32_t* sptPar,
                             uint32_t* adjk, float* kap, float* ksum, float* kap0,
                             hipStream_t st) {
    if (nadj <= 0 || V <= 0) return hipSuccess;
    Tmp<unsigned long long> k0, k1;
    Tmp<uint32_t> i0, i1;
    Tmp<unsigned char> tmp;
    PCHK(k0.alloc(nadj));
    PCHK(k1.alloc(nadj));
    PCHK(i0.alloc(nadj));
    PCHK(i1.alloc(nadj));
    const unsigned g = std::max(grid_for(V), (unsigned)std::min<int64_t>((hs.nseg + 3) / 4, 256 * 64));
    hipLaunchKernelGGL(kap_key_kernel, dim3(g), dim3(kPB), 0, st, V, hs, rowptr, adj, pot, k0.p,
                       i0.p);
    PCHK(hipGetLastError());
    const int endbit = 32 + bitlen((uint64_t)V);
    size_t tb = 0;
    PCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0.p, k1.p, i0.p, i1.p, (int)nadj, 0,
                                            endbit, st));
    PCHK(tmp.alloc(tb));
    PCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k0.p, k1.p, i0.p, i1.p, (int)nadj, 0, endbit,
                                            st));
    hipLaunchKernelGGL(kap_gather_kernel, dim3(grid_for(nadj)), dim3(kPB), 0, st, nadj, k1.p, i1.p,
                       adj, sptPar, adjk, kap);
    PCHK(hipGetLastError());
    hipLaunchKernelGGL(kap_probe_kernel, dim3(grid_for(V)), dim3(kPB), 0, st, V, rowptr, kap, ksum,
                       kap0);
    PCHK(hipGetLastError());
    return hipStreamSynchronize(st);
}

hipError_t prep_replay_csr(int64_t V, int64_t E, int directed, const int32_t* eu,
                           const int32_t* ev, const double* elat, const double* eloss,
                           const uint32_t* inv, const double* pot, uint32_t* rowptr, uint4* rec,
                           uint32_t* own, double2* hop, int64_t* nrec, hipStream_t st) {
    const int64_t n = directed ? E : 2 * E;
    Tmp<unsigned long long> k0, k1;
    Tmp<uint32_t> v0, v1, start, gpos, cnt;
    Tmp<unsigned char> tmp;
    PCHK(k0.alloc(n));
    PCHK(k1.alloc(n));
    PCHK(v0.alloc(n));
    PCHK(v1.alloc(n));
    PCHK(start.alloc(n));
    PCHK(gpos.alloc(n));
    PCHK(cnt.alloc(V + 1));
    const unsigned long long sentinel = (unsigned long long)V << 32;
    hipLaunchKernelGGL(rp_entry_kernel, dim3(grid_for(E)), dim3(kPB), 0, st, E, directed, eu, ev,
                       inv, k0.p, v0.p, sentinel);
    PCHK(hipGetLastError());
    const int endbit = 32 + bitlen((uint64_t)V);
    size_t tb = 0, tb2 = 0, tb3 = 0;
    PCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0.p, k1.p, v0.p, v1.p, (int)n, 0, endbit,
                                            st));
    PCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, start.p, gpos.p, (int)n, st));
    PCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb3, cnt.p, rowptr, (int)(V + 1), st));
    PCHK(tmp.alloc(std::max(tb, std::max(tb2, tb3))));
    PCHK(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, k0.p, k1.p, v0.p, v1.p, (int)n, 0, endbit,
                                            st));
    PCHK(hipMemsetAsync(cnt.p, 0, sizeof(uint32_t) * (size_t)(V + 1), st));
    hipLaunchKernelGGL(rp_group_kernel, dim3(grid_for(n)), dim3(kPB), 0, st, n, k1.p, sentinel,
                       start.p, cnt.p);
    PCHK(hipGetLastError());
    PCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb2, start.p, gpos.p, (int)n, st));
    PCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb3, cnt.p, rowptr, (int)(V + 1), st));
    hipLaunchKernelGGL(rp_fill_kernel, dim3(grid_for(n)), dim3(kPB), 0, st, n, k1.p, v1.p, start.p,
                       gpos.p, directed, inv, pot, elat, eloss, rec, own, hop);
    PCHK(hipGetLastError());
    uint32_t nr = 0;
    PCHK(hipMemcpyAsync(&nr, rowptr + V, 4, hipMemcpyDeviceToHost, st));
    PCHK(hipStreamSynchronize(st));
    *nrec = nr;
    return hipSuccess;
}

hipError_t preload_prep_module() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)prep_degree_kernel);
}

}  // namespace shdtopo
