// topo_kernels.hip -- CDNA4 (gfx950) kernels of the routing engine.
//
//   sssp_rows_kernel            replaces igraph_get_shortest_paths_dijkstra
//                               (src/topology/shd-topology.c:753-787) + the per-target helper
//                               (shd-topology.c:561-671, 808-823): one persistent workgroup per
//                               SSSP slot runs a near-far (delta-stepping) label-correcting SSSP
//                               for one source at a time, then derives igraph's parents with the
//                               argmin (d[u]) rule and walks them to produce
//                               latency (== dist, bit-exact), reliability (reference product
//                               order) and hop count for every attached target.
//   pair_table_complete_kernel  replaces _topology_lookupPath (shd-topology.c:835-873).
//   packet_route_kernel         replaces worker_schedulePacket (src/engine/shd-worker.c:332-370)
//                               for a whole scheduler window.
//
// f64 arithmetic: every latency add is a single IEEE add (no contraction: built with
// -ffp-contract=off, and there is no multiply to fuse with); reliability multiplies happen in the
// reference order.  Distances are the unique monotone-rounding fixpoint, so any correct
// label-correcting order yields the same bits as igraph's heap order.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "topo_dev_common.h"

namespace shdtopo {

namespace {

using namespace dev;

#ifndef SHD_RING_SLOTS
#define SHD_RING_SLOTS 48
#endif
constexpr int kRingSlots = SHD_RING_SLOTS;  // buckets in the window (<= 64: one ballot scans them)
static_assert(kRingSlots >= 2 && kRingSlots <= 64, "window slots must fit one wave ballot");

struct Lds {
    uint32_t off[kSsspBlock + 4];
    uint32_t rs[kSsspBlock];
    uint32_t vx[kSsspBlock];
    double val[kSsspBlock];
    uint32_t wave[kSsspBlock / 64];
    uint32_t rtail[kRingSlots];  // entries pushed into each bucket of the window
    uint32_t qtail;
    uint32_t otail;    // entries in the overflow pile
    uint32_t src_idx;
    uint32_t fover;    // a window slot / the overflow pile overflowed: scanning buckets from now on
    uint32_t nover;    // a near queue overflowed since the last bucket change: re-expand the bucket
    uint32_t pad;
    unsigned long long dmin;
    unsigned long long fmin;  // scanning mode: lower bound of the unexpanded distances above cb
    unsigned long long omin;  // lower bound of the keys in the overflow pile
};
constexpr size_t kLdsCtrlBytes = (sizeof(Lds) + 15) / 16 * 16;
constexpr uint32_t kParHubs = 2048;         // hubs whose parent is tracked during the SSSP
constexpr size_t kSsspMaxLds = 160 * 1024;  // LDS of one CU, shared by its SSSP workgroups
#ifndef SHD_RELAX_UNROLL
#define SHD_RELAX_UNROLL 4
#endif
constexpr int kRelaxUnroll = SHD_RELAX_UNROLL;
// Tail relaxations: a plain pre-check load, then a no-return atomicMin when the candidate is
// smaller; the push is decided on the pre-check (a lost race pushes a stale entry, skipped or
// re-expanded harmlessly), so no returning atomic sits on the relaxation's dependency chain.
#ifndef SHD_TAIL_NORET
#define SHD_TAIL_NORET 1
#endif
#ifndef SHD_NT_DIST
#define SHD_NT_DIST 0
#endif
#ifndef SHD_STALE_FIRST
#define SHD_STALE_FIRST 1
#endif

// Dynamic LDS after the control block: the near-queue dedupe bitmap nbits[hw], parent-tie bits
// tbits[pw], parent hints hpar[P] (u32), then the hub distance words hd[H] (u64).
struct LdsLayout {
    uint32_t hw, pw;
    size_t nbits, tbits, hpar, hd, bytes;
};
__host__ __device__ inline LdsLayout lds_layout(uint32_t H, uint32_t P) {
    LdsLayout l;
    l.hw = (H + 31) / 32;
    l.pw = (P + 31) / 32;
    l.nbits = kLdsCtrlBytes;
    l.tbits = l.nbits + 4 * (size_t)l.hw;
    l.hpar = l.tbits + 4 * (size_t)l.pw;
    l.hd = (l.hpar + 4 * (size_t)P + 7) & ~(size_t)7;
    l.bytes = l.hd + 8 * (size_t)H;
    return l;
}

// Wave-aggregated queue append: one LDS atomic per wave instead of one per lane.
__device__ __forceinline__ void wave_push(bool pred, uint32_t val, uint32_t* q, uint32_t* lds_tail,
                                          uint32_t cap, unsigned long long* stats) {
    unsigned long long m = __ballot(pred);
    if (m == 0ull) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(lds_tail, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) {
        uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (pos < cap) q[pos] = val;
        else atomicOr(&stats[ST_OVERFLOW], 1ull);
    }
}

__device__ __forceinline__ void wave_push64(bool pred, unsigned long long val,
                                            unsigned long long* q, uint32_t* lds_tail,
                                            uint32_t cap, uint32_t* lds_over,
                                            uint32_t code = 1u) {
    unsigned long long m = __ballot(pred);
    if (m == 0ull) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(lds_tail, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) {
        uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (pos < cap) q[pos] = val;
        else atomicOr(lds_over, code);
    }
}

// Far-pile entry: the high word of the f64 key's bit pattern over the vertex id.  For d >= 0
// the bit pattern orders like the value, so hi32 truncation gives a lower bound of the key
// (key_lb(e) <= the distance the vertex had when the entry was pushed).
__device__ __forceinline__ unsigned long long far_entry(unsigned long long dbits, uint32_t v) {
    return (dbits & 0xFFFFFFFF00000000ull) | (unsigned long long)v;
}
__device__ __forceinline__ double far_key_lb(unsigned long long e) {
    return bits2d(e & 0xFFFFFFFF00000000ull);
}

// Block-wide exclusive scan of one u32 per thread; *total receives the sum.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t x, Lds& L, uint32_t* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int NW = kSsspBlock / 64;
    uint32_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) L.wave[wid] = v;
    __syncthreads();
    if (wid == 0) {
        uint32_t w = lane < NW ? L.wave[lane] : 0u;
#pragma unroll
        for (int o = 1; o < NW; o <<= 1) {
            uint32_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < NW) L.wave[lane] = w;
    }
    __syncthreads();
    uint32_t base = wid ? L.wave[wid - 1] : 0u;
    *total = L.wave[NW - 1];
    __syncthreads();
    return base + v - x;
}

// Load-balanced expansion of the adjacency lists of queue Q[0..nq): the queue is taken in chunks
// of kSsspBlock vertices; a block scan of their degrees flattens the chunk's edges and every
// lane takes edges (tid, tid+B, ...) and finds its vertex by binary search in LDS.  Hubs with
// 10^5 edges are spread over the whole workgroup.  VF decides per vertex whether to expand and
// the f64 value carried with it; EF handles one edge (vertex, value, adjacency slot, valid).
template <class VF, class EF>
__device__ __forceinline__ void expand_queue(const uint32_t* Q, uint32_t nq, const DevCSR& g,
                                             Lds& L, VF&& vf, EF&& ef) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t base = 0; base < nq; base += kSsspBlock) {
        const uint32_t cnt = min((uint32_t)kSsspBlock, nq - base);
        uint32_t deg = 0;
        if (tid < cnt) {
            uint32_t v = Q[base + tid];
            double val;
            if (vf(v, val)) {
                uint32_t r0 = g.rowptr[v], r1 = g.rowptr[v + 1];
                deg = r1 - r0;
                L.rs[tid] = r0;
            } else {
                L.rs[tid] = 0;
            }
            L.vx[tid] = v;
            L.val[tid] = val;
        }
        uint32_t total;
        uint32_t off = block_excl_scan(deg, L, &total);
        if (tid < cnt) L.off[tid] = off;
        if (tid == 0) L.off[cnt] = total;
        __syncthreads();
        const uint32_t lane = tid & 63;
        for (uint32_t eb = tid - lane; eb < total; eb += kSsspBlock) {
            const uint32_t e = eb + lane;
            const bool valid = e < total;
            int lo = 0;
            if (valid) {
                int hi = (int)cnt - 1;
                while (lo < hi) {
                    int mid = (lo + hi + 1) >> 1;
                    if (L.off[mid] <= e) lo = mid; else hi = mid - 1;
                }
            }
            const uint32_t j = valid ? L.rs[lo] + (e - L.off[lo]) : 0u;
            ef(L.vx[lo], L.val[lo], j, valid);
        }
        __syncthreads();
    }
}


// Hot-distance cache: after the degree relabel the first H vertex ids are the hubs, which receive
// most relaxations of a power-law graph.  Their distance words live in LDS for the whole SSSP of
// a source (the authoritative copy: LDS atomics, no DRAM traffic); the tail stays in HBM.
struct DistView {
    unsigned long long* hd;    // LDS, H words
    unsigned long long* dist;  // HBM, V words (words < H unused while the source runs)
    uint32_t* nbits;           // LDS: hub already in the next near queue (this iteration)
    uint32_t* hpar;            // LDS: vertex whose relaxation last lowered hub v (v < kParHubs)
    uint32_t* tbits;           // LDS: a relaxation tied hub v's current distance (v < kParHubs)
    uint32_t H;
    uint32_t P;                // hubs with parent hints (<= kParHubs)
    __device__ __forceinline__ unsigned long long get(uint32_t v) const {
        return v < H ? hd[v] : ld_l2_u64(&dist[v]);
    }
};

// The buckets of one source.  The window holds the kRingSlots buckets [wbase, wbase + kRingSlots)
// in fixed slots; later buckets go to the overflow pile, which a refill re-sorts into the window
// once the window is used up.  cb = the bucket being settled.
struct Buckets {
    double inv_delta;
    uint32_t cb, wbase;
    unsigned long long* ring;  // kRingSlots slots of slot_cap entries
    uint32_t slot_cap;
    ulonglong2* over;          // overflow pile (current buffer): {exact key bits, vertex}
    uint32_t ocap;
};

__device__ __forceinline__ void wave_push_over(bool pred, unsigned long long key, uint32_t v,
                                               ulonglong2* q, uint32_t* lds_tail, uint32_t cap,
                                               uint32_t* lds_over, uint32_t code) {
    unsigned long long m = __ballot(pred);
    if (m == 0ull) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(lds_tail, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) {
        const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (pos < cap) q[pos] = make_ulonglong2(key, (unsigned long long)v);
        else atomicOr(lds_over, code);
    }
}

// Window push: lanes may target different slots; one LDS atomic per (wave, slot).
__device__ __forceinline__ void ring_push(bool pred, uint32_t slot, unsigned long long val,
                                          const Buckets& B, Lds& L) {
    unsigned long long m = __ballot(pred);
    const int lane = threadIdx.x & 63;
    while (m) {
        const int leader = __ffsll((long long)m) - 1;
        const uint32_t s = __shfl(slot, leader, 64);
        const bool mine = pred && slot == s;
        const unsigned long long mm = __ballot(mine);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&L.rtail[s], (uint32_t)__popcll(mm));
        base = __shfl(base, leader, 64);
        if (mine) {
            const uint32_t pos = base + (uint32_t)__popcll(mm & ((1ull << lane) - 1ull));
            if (pos < B.slot_cap) B.ring[(size_t)s * B.slot_cap + pos] = val;
            else atomicOr(&L.fover, 2u);
        }
        m &= ~mm;
    }
}

// Near-phase relaxation of queue Q: the load-balanced chunking of expand_queue, with U edges in
// flight per lane: U (col, wt) loads, then the U tail pre-checks, then the LDS atomics / no-return
// HBM atomics, then the pushes.  An improvement to bucket b goes to the near queue (b <= cb), the
// window slot of b, or the overflow pile.
//   Far entries: pushed only when the improvement moves the vertex to an EARLIER bucket than the
//   value it had (hubs: the LDS atomic's return; tails: the pre-check, whose staleness can only
//   overstate the old bucket).  Invariant: every unexpanded vertex with bucket(d) > cb has an
//   entry in exactly bucket(d), so a same-bucket improvement needs none.  A window-slot entry is
//   stale once its vertex has moved to a bucket < cb (win); a near entry once its vertex's
//   distance dropped below the entry's key (the high word rides in the entry).
//   scan: scanning mode after an overflow (near pushes deduplicated by stamp, far improvements
//   only lower L.fmin).
template <int U, bool EV>
__device__ __forceinline__ void relax_queue(const unsigned long long* Q, uint32_t nq,
                                            const DevCSR& g, Lds& L, const DistView& D,
                                            uint32_t* stamp, bool scan, bool win,
                                            unsigned long long* nxt, const Buckets& B,
                                            uint32_t it, uint32_t ncap,
                                            unsigned long long& relax,
                                            unsigned long long* ev) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    const uint32_t wend = B.wbase + (uint32_t)kRingSlots;
    for (uint32_t base = 0; base < nq; base += kSsspBlock) {
        const uint32_t cnt = min((uint32_t)kSsspBlock, nq - base);
        uint32_t deg = 0;
        if (tid < cnt) {
            // an entry of a non-deduplicating push carries the high word of its distance; a
            // later (smaller) push of the same vertex supersedes it, so an entry whose word is
            // above the current distance's is stale and expands nothing (entries of deduplicated
            // pushes carry 0)
            const unsigned long long e = Q[base + tid];
            const uint32_t v = (uint32_t)e;
#if SHD_STALE_FIRST
            // the distance decides staleness before the row bounds are fetched: a stale entry
            // costs one read instead of two
            const unsigned long long dv = D.get(v);
            const bool stale = win ? bucket_of(bits2d(dv), B.inv_delta) < B.cb
                                   : (dv >> 32) < (e >> 32);
            uint32_t r0 = 0, r1 = 0;
            if (!stale) {
                r0 = g.rowptr[v];
                r1 = g.rowptr[v + 1];
            }
#else
            const uint32_t r0 = g.rowptr[v], r1 = g.rowptr[v + 1];
            const unsigned long long dv = D.get(v);
            const bool stale = win ? bucket_of(bits2d(dv), B.inv_delta) < B.cb
                                   : (dv >> 32) < (e >> 32);
#endif
            deg = stale ? 0u : r1 - r0;
            if constexpr (EV) ev[7] += stale ? 1ull : 0ull;
            L.rs[tid] = r0;
            L.vx[tid] = v;
            L.val[tid] = bits2d(dv);
        }
        uint32_t total;
        const uint32_t off = block_excl_scan(deg, L, &total);
        if (tid < cnt) L.off[tid] = off;
        if (tid == 0) L.off[cnt] = total;
        relax += total;  // uniform: every adjacency entry of the chunk is relaxed once
        __syncthreads();
        for (uint32_t eb = tid - lane; eb < total; eb += kSsspBlock * U) {
            // Loads are issued unconditionally (an idle lane reads entry 0 / word 0 and discards
            // it): a load inside a divergent branch is waited for inside that branch, which
            // would serialise the U round trips.
            uint32_t n[U], from[U];
            unsigned long long ab[U];
            bool valid[U];
            AdjRec rec[U];
            int los[U];
#pragma unroll
            for (int u = 0; u < U; u++) {  // U searches, U record loads in flight
                const uint32_t e = eb + (uint32_t)u * kSsspBlock + lane;
                valid[u] = e < total;
                int lo = 0;
                if (valid[u]) {
                    int hi = (int)cnt - 1;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (L.off[mid] <= e) lo = mid; else hi = mid - 1;
                    }
                }
                los[u] = lo;
                const uint32_t j = valid[u] ? L.rs[lo] + (e - L.off[lo]) : 0u;
                rec[u] = adj_rec(g, j);
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const double w = __hiloint2double((int)rec[u].c, (int)rec[u].b);
                const double a = __dadd_rn(L.val[los[u]], w);
                n[u] = valid[u] ? rec[u].a : 0u;
                from[u] = L.vx[los[u]];
                ab[u] = valid[u] ? d2bits(a) : ~0ull;
            }
            unsigned long long cur[U];
#pragma unroll
            for (int u = 0; u < U; u++) {  // tail pre-check (plain load: stale = larger = safe)
                const bool t = valid[u] && n[u] >= D.H;
#if SHD_NT_DIST
                const unsigned long long x = __builtin_nontemporal_load(&D.dist[t ? n[u] : 0u]);
#else
                const unsigned long long x = D.dist[t ? n[u] : 0u];
#endif
                cur[u] = t ? x : 0ull;
            }
            bool imp[U];
            unsigned long long hold[U];  // hubs: the exact previous value (bucket dedupe below)
#pragma unroll
            for (int u = 0; u < U; u++) {
                imp[u] = false;
                hold[u] = kInfBits;
                if (valid[u] && n[u] < D.H) {
                    const unsigned long long old = atomicMin(&D.hd[n[u]], ab[u]);
                    hold[u] = old;
                    imp[u] = ab[u] < old;
                    if (n[u] < D.P) {  // parent hint for the heaviest rows (see epilogue)
                        if (imp[u]) D.hpar[n[u]] = from[u];
                        else if (ab[u] == old) atomicOr(&D.tbits[n[u] >> 5], 1u << (n[u] & 31));
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++)
                if (ab[u] < cur[u]) {
#if SHD_TAIL_NORET
                    (void)atomicMin(&D.dist[n[u]], ab[u]);
                    imp[u] = true;
#else
                    imp[u] = ab[u] < atomicMin(&D.dist[n[u]], ab[u]);
#endif
                }
            unsigned long long om = kInfBits, fm = kInfBits;
#pragma unroll
            for (int u = 0; u < U; u++) {
                bool pN = false, pR = false, pO = false;
                const uint32_t b = imp[u] ? bucket_of(bits2d(ab[u]), B.inv_delta) : 0u;
                if (imp[u]) {
                    if (b <= B.cb) {
                        if (n[u] < D.H) {  // hub: dedupe in LDS, no memory-side atomic
                            const uint32_t bit = 1u << (n[u] & 31);
                            pN = (atomicOr(D.nbits + (n[u] >> 5), bit) & bit) == 0u;
                        } else {
                            // no dedupe: every strict improvement pushes (its value rides
                            // along and stale entries are skipped at expansion).  In scanning
                            // mode the source deduplicates per iteration (<= V entries).
                            pN = !scan || atomicExch(&stamp[n[u]], it) != it;
                        }
                    } else if (scan) {
                        fm = ab[u] < fm ? ab[u] : fm;
                    } else if (b < bucket_of(bits2d(n[u] < D.H ? hold[u] : cur[u]),
                                             B.inv_delta)) {
                        if (b < wend) {
                            pR = true;
                        } else {
                            pO = true;
                            om = ab[u] < om ? ab[u] : om;
                        }
                    }
                }
                // hub near pushes and scanning-mode pushes are deduplicated: key 0 (never stale)
                wave_push64(pN, far_entry((n[u] < D.H || scan) ? 0ull : ab[u], n[u]), nxt,
                            &L.qtail, ncap, &L.nover, 1u);
                ring_push(pR, b - B.wbase, far_entry(ab[u], n[u]), B, L);
                wave_push_over(pO, ab[u], n[u], B.over, &L.otail, B.ocap, &L.fover, 4u);
                if constexpr (EV) {
                    ev[1] += (valid[u] && n[u] >= D.H) ? 1ull : 0ull;
                    ev[2] += (imp[u] && n[u] >= D.H) ? 1ull : 0ull;
                    ev[6] += (valid[u] && n[u] >= D.H &&
                              bucket_of(bits2d(cur[u]), B.inv_delta) < B.cb) ? 1ull : 0ull;
                }
            }
            if (__ballot(om != kInfBits || fm != kInfBits)) {
                om = wave_min_u64(om);
                fm = wave_min_u64(fm);
                if (lane == 0 && om != kInfBits) atomicMin(&L.omin, om);
                if (lane == 0 && fm != kInfBits) atomicMin(&L.fmin, fm);
            }
        }
        // the no-return atomics and queue stores of this wave complete before any wave reads
        // the distances or queues after the barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

}  // namespace

template <bool EV>
__global__ void __launch_bounds__(kSsspBlock, 4)
sssp_rows_kernel(DevCSR g, SlotWs ws, const uint32_t* __restrict__ sources, int nsrc,
                 const uint32_t* __restrict__ targets, int A, double delta, uint32_t hubs,
                 uint32_t parhubs, uint32_t far_cap, uint32_t near_cap,
                 double2* __restrict__ out_lr, uint16_t* __restrict__ out_hops,
                 double* __restrict__ out_rowmin, unsigned long long* __restrict__ stats) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    Lds& L = *reinterpret_cast<Lds*>(smem);
    const int slot = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const int64_t V = ws.V;
    DistView D;
    const LdsLayout lay = lds_layout(hubs, parhubs);
    const uint32_t hw = lay.hw;
    D.nbits = reinterpret_cast<uint32_t*>(smem + lay.nbits);
    D.tbits = reinterpret_cast<uint32_t*>(smem + lay.tbits);
    D.hpar = reinterpret_cast<uint32_t*>(smem + lay.hpar);
    D.hd = reinterpret_cast<unsigned long long*>(smem + lay.hd);
    D.dist = ws.dist + (size_t)slot * V;
    D.H = hubs;
    D.P = parhubs;
    unsigned long long* dist = D.dist;
    uint32_t* stamp = ws.stamp + (size_t)slot * V;
    unsigned long long* qa = ws.qa + (size_t)slot * kNearPerVertex * V;
    unsigned long long* qb = ws.qb + (size_t)slot * kNearPerVertex * V;
    const size_t ring_all = (size_t)kRingPerVertex * (size_t)V;
    const size_t over_all = (size_t)kOverPerVertex * (size_t)V;
    ulonglong2* over0 = reinterpret_cast<ulonglong2*>(ws.over) + (size_t)slot * 2 * over_all;
    ulonglong2* over1 = over0 + over_all;
    uint32_t* fscr = reinterpret_cast<uint32_t*>(over0);  // parent-pass scratch queue (u32)
    unsigned long long* best = ws.best + (size_t)slot * V;
    uint32_t* cntc = ws.cnt + (size_t)slot * V;
    uint32_t* bslot = ws.bslot + (size_t)slot * V;
    unsigned long long* memo = ws.memo + (size_t)slot * V;
    uint32_t* par = ws.par + (size_t)slot * V;
    uint32_t* pbuf = ws.pathbuf + (size_t)slot * kMaxHops * kSsspBlock;
    uint32_t* ctr = ws.counters + (size_t)slot * 4;
    const uint32_t cap = (uint32_t)V;
    // near queues hold kNearPerVertex * V entries; deduplicated pushes (scanning mode) never
    // exceed V.  near_cap / far_cap only shrink the non-deduplicated queues (tests force the
    // overflow fallback with them).
    const uint32_t ncap = (uint32_t)(kNearPerVertex * V);
    const uint32_t ncap_free = (near_cap > 0 && near_cap < ncap) ? near_cap : ncap;
    Buckets B;
    B.inv_delta = 1.0 / delta;
    B.ring = ws.ring + (size_t)slot * ring_all;
    B.slot_cap = (uint32_t)(ring_all / kRingSlots);
    B.ocap = (uint32_t)over_all;
    if (far_cap > 0) {
        B.slot_cap = min(B.slot_cap, far_cap);
        B.ocap = min(B.ocap, far_cap);
    }

    // slot-persistent epoch counters (never reset, so stamp/memo need no clearing)
    uint32_t iter = ctr[0], mep = ctr[2];
    unsigned long long relax_local = 0;
    unsigned long long nfarscan = 0;
    unsigned long long ev[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // per-lane (EV builds only)
    unsigned long long ev0 = 0, ev3 = 0, ev4 = 0, ev5 = 0;  // uniform across the workgroup
    unsigned long long t_split = 0;
    unsigned long long t_init = 0, t_sssp = 0, t_par = 0, t_tgt = 0, n_near = 0, n_split = 0;
    unsigned long long tk = wall_clock64();

    for (;;) {
        if (tid == 0) L.src_idx = (uint32_t)atomicAdd(&stats[ST_DEQUEUE], 1ull);
        __syncthreads();
        const uint32_t s_idx = L.src_idx;
        __syncthreads();
        if (s_idx >= (uint32_t)nsrc) break;
        const uint32_t src = sources[s_idx];
        tk = wall_clock64();

        // ---------------- SSSP (delta-stepping: near queue + bucket window + overflow) -------
        for (uint32_t v = tid; v < D.H; v += kSsspBlock) D.hd[v] = kInfBits;
        for (uint32_t w = tid; w < lay.pw; w += kSsspBlock) D.tbits[w] = 0u;
        for (uint32_t k = tid; k < (uint32_t)kRingSlots; k += kSsspBlock) L.rtail[k] = 0u;
        for (int64_t v = (int64_t)D.H + tid; v < V; v += kSsspBlock) dist[v] = kInfBits;
        __syncthreads();
        { unsigned long long t = wall_clock64(); t_init += t - tk; tk = t; }
        iter++;
        if (tid == 0) {
            L.fover = 0u;
            L.nover = 0u;
            if (src < D.H) D.hd[src] = 0ull; else dist[src] = 0ull;
            qa[0] = far_entry(0ull, src);
            stamp[src] = iter;
            L.otail = 0;
            L.omin = kInfBits;
            L.fmin = kInfBits;
        }
        __syncthreads();
        B.cb = 0;
        B.wbase = 0;
        B.over = over0;
        ulonglong2* over_alt = over1;
        bool win = false;  // inq is a window slot (bucket-based stale test)
        const unsigned long long* inq = qa;  // near-phase input: a near queue or a window slot
        unsigned long long* qnxt = qb;       // near-phase output (never aliases inq)
        uint32_t nq = 1;
        uint32_t guard = 0;
        constexpr int FU = 4;  // entries per lane per chunk in the streaming passes
        unsigned long long tsplit0 = 0;
        for (;;) {
            if (tsplit0) {
                t_split += wall_clock64() - tsplit0;
                tsplit0 = 0;
            }
            while (nq > 0) {
                iter++;
                if (tid == 0) L.qtail = 0;
                for (uint32_t w = tid; w < hw; w += kSsspBlock) D.nbits[w] = 0u;
                __syncthreads();
                ev0 += nq;
                const bool scan = L.fover != 0u;
                relax_queue<kRelaxUnroll, EV>(inq, nq, g, L, D, stamp, scan, win, qnxt, B, iter,
                                              scan ? ncap : ncap_free, relax_local, ev);
                // relax_queue ends with a barrier
                nq = min(L.qtail, ncap);
                win = false;
                inq = qnxt;
                qnxt = (qnxt == qa) ? qb : qa;
                n_near++;
                if (++guard > 4000000u) {
                    if (tid == 0) atomicOr(&stats[ST_OVERFLOW], 2ull);
                    nq = 0;
                }
                __syncthreads();
            }
            if (guard > 4000000u) break;
            tsplit0 = wall_clock64();
            const bool nov = L.nover != 0u;
            if (L.fover != 0u || nov) {
                // Scanning mode: a queue overflowed (entries were lost), so for the rest of this
                // source the next bucket is found by classifying every vertex by its distance.
                // Every unexpanded vertex is in a bucket > cb -- unless a near queue overflowed
                // since the last bucket change: then the whole bucket cb is expanded again
                // (re-expansion is harmless for a label-correcting SSSP).  L.fmin is exact after
                // the first scanning pass (bit 64 of fover), a lower bound before.
                const bool exact = (L.fover & 64u) != 0u;
                const unsigned long long fmb = L.fmin;
                if (!nov && exact && fmb == kInfBits) break;
                uint32_t nb = B.cb + 1;
                if (exact && fmb != kInfBits) nb = max(nb, bucket_of(bits2d(fmb), B.inv_delta));
                const uint32_t lob = nov ? B.cb : B.cb + 1;
                iter++;
                __syncthreads();
                if (tid == 0) {
                    L.qtail = 0;
                    L.fmin = kInfBits;
                    L.nover = 0u;
                    L.fover |= 64u;
                }
                __syncthreads();
                for (uint32_t base = 0; base < (uint32_t)V; base += kSsspBlock * FU) {
                    unsigned long long km = kInfBits;
#pragma unroll
                    for (int u = 0; u < FU; u++) {
                        const uint32_t v = base + (uint32_t)u * kSsspBlock + tid;
                        bool pN = false;
                        if (v < (uint32_t)V) {
                            const unsigned long long b = D.get(v);
                            const uint32_t k = bucket_of(bits2d(b), B.inv_delta);
                            pN = b != kInfBits && k >= lob && k <= nb;
                            if (b != kInfBits && k > nb && b < km) km = b;
                        }
                        wave_push64(pN, far_entry(0ull, v), qnxt, &L.qtail, ncap, &L.nover, 32u);
                    }
                    km = wave_min_u64(km);
                    if ((tid & 63) == 0 && km != kInfBits) atomicMin(&L.fmin, km);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                nq = min(L.qtail, ncap);
                inq = qnxt;
                qnxt = (qnxt == qa) ? qb : qa;
                B.cb = nb;
                n_split++;
                __syncthreads();
                continue;
            }
            // next non-empty bucket of the window after cb (every wave scans the slot tails)
            int s = -1;
            {
                const int lane = (int)(tid & 63);
                const int lo_slot = (int)B.cb - (int)B.wbase + 1;  // 0 right after a refill
                const bool ne = lane < kRingSlots && lane >= lo_slot && L.rtail[lane] > 0u;
                const unsigned long long m = __ballot(ne);
                s = m ? __ffsll((long long)m) - 1 : -1;
            }
            if (s >= 0) {
                const uint32_t n = min(L.rtail[s], B.slot_cap);
                __syncthreads();
                // the slot receives no pushes before the next refill (only buckets > cb do)
                if (tid == 0) L.rtail[s] = 0u;
                ev3 += n;
                B.cb = B.wbase + (uint32_t)s;
                inq = B.ring + (size_t)s * B.slot_cap;
                win = true;
                nq = n;
                n_split++;
                continue;
            }
            // window used up: refill it from the overflow pile (or the source is done).  The
            // window restarts at the overflow's smallest key; an entry goes to the window slot
            // of its exact key's bucket, or back to the pile.  No distance reads.
            const uint32_t no = min(L.otail, B.ocap);
            if (no == 0) break;
            {
                const uint32_t kb = bucket_of(bits2d(L.omin), B.inv_delta);
                const uint32_t wb = max(B.cb + 1, kb);
                const uint32_t we = wb + (uint32_t)kRingSlots;
                __syncthreads();
                if (tid == 0) {
                    L.otail = 0;
                    L.omin = kInfBits;
                }
                __syncthreads();
                Buckets R = B;
                R.wbase = wb;
                for (uint32_t base = 0; base < no; base += kSsspBlock * FU) {
                    unsigned long long k2 = kInfBits;
#pragma unroll
                    for (int u = 0; u < FU; u++) {
                        const uint32_t i = base + (uint32_t)u * kSsspBlock + tid;
                        const ulonglong2 e = i < no ? B.over[i] : make_ulonglong2(0ull, 0ull);
                        const uint32_t b = max(bucket_of(bits2d(e.x), B.inv_delta), wb);
                        const bool mv = i < no && b < we;
                        const bool kp = i < no && !mv;
                        if (kp) k2 = e.x < k2 ? e.x : k2;
                        ring_push(mv, b - wb, far_entry(e.x, (uint32_t)e.y), R, L);
                        wave_push_over(kp, e.x, (uint32_t)e.y, over_alt, &L.otail, B.ocap,
                                       &L.fover, 8u);
                    }
                    k2 = wave_min_u64(k2);
                    if ((tid & 63) == 0 && k2 != kInfBits) atomicMin(&L.omin, k2);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                ev4 += no;
                { ulonglong2* t = B.over; B.over = over_alt; over_alt = t; }
                B.wbase = wb;
                B.cb = wb - 1;
                nq = 0;
            }
        }

        nfarscan += L.fover ? 1u : 0u;
        if (tid == 0 && (L.fover | L.nover)) atomicOr(&stats[ST_OVERSITE], (unsigned long long)(L.fover | L.nover));
        { unsigned long long t = wall_clock64(); t_sssp += t - tk; tk = t; }
        // ---------------- parents for the target chains (argmin d[u]) ----------
        uint32_t* pcur = reinterpret_cast<uint32_t*>(qa);  // u32 views of the near queues
        uint32_t* pnxt = reinterpret_cast<uint32_t*>(qb);
        // One adjacency pass per chain level finds min d[u] over the candidates
        // fl(d[u] + w) == d[v] and counts them; only vertices with more than one candidate get a
        // second pass that counts the candidates AT the minimum and keeps the lowest slot.
        mep++;
        const unsigned long long mtag = (unsigned long long)mep << 32;
        iter++;
        if (tid == 0) L.qtail = 0;
        __syncthreads();
        for (uint32_t kb = 0; kb < (uint32_t)A; kb += kSsspBlock) {
            const uint32_t k = kb + tid;
            bool p = false;
            uint32_t t = 0;
            if (k < (uint32_t)A) {
                t = targets[k];
                p = (t != src) && (atomicExch(&stamp[t], iter) != iter);
                if (p) { best[t] = kInfBits; cntc[t] = 0; bslot[t] = 0xFFFFFFFFu; }
            }
            wave_push(p, t, pcur, &L.qtail, cap, stats);
        }
        __syncthreads();
        uint32_t nF = min(L.qtail, cap);
        __syncthreads();
        while (nF > 0) {
            ev5 += nF;
            // Heavy hubs first: the SSSP recorded which vertex last lowered each of the first
            // kParHubs hubs and whether any relaxation tied its value.  Every candidate u of v
            // relaxes v with fl(d[u]+w) == d[v] when u is expanded at its final distance, so
            // "no tie seen" + "the recorded u is a candidate" means u is the only candidate:
            // the igraph parent, found without scanning the hub's (up to 10^5-entry) row.
            // Anything else falls back to the exact scan below.
            if (tid == 0) L.qtail = 0;
            __syncthreads();
            for (uint32_t ib = 0; ib < nF; ib += kSsspBlock) {
                const uint32_t i = ib + tid;
                bool scan = false;
                uint32_t v = 0;
                if (i < nF) {
                    v = pcur[i];
                    scan = true;
                    if (g.rows_sorted && v < D.P && v < D.H &&
                        !((D.tbits[v >> 5] >> (v & 31)) & 1u)) {
                        const uint32_t u = D.hpar[v];
                        if (u < (uint32_t)V) {
                            uint32_t lo = g.rowptr[u], hi = g.rowptr[u + 1];
                            while (lo < hi) {  // rows are sorted by neighbour
                                const uint32_t mid = (lo + hi) >> 1;
                                if (adj_col(g, mid) < v) lo = mid + 1; else hi = mid;
                            }
                            if (lo < g.rowptr[u + 1] && adj_col(g, lo) == v) {
                                uint32_t c;
                                double w;
                                adj_load(g, lo, c, w);
                                if (__dadd_rn(bits2d(D.get(u)), w) == bits2d(D.get(v))) {
                                    memo[v] = mtag | (unsigned long long)lo;  // slot in u's row
                                    par[v] = u;
                                    scan = false;
                                }
                            }
                        }
                    }
                }
                wave_push(scan, v, fscr, &L.qtail, cap, stats);
            }
            __syncthreads();
            const uint32_t nS = min(L.qtail, cap);
            __syncthreads();
            expand_queue(
                fscr, nS, g, L,
                [&](uint32_t v, double& val) {
                    val = bits2d(D.get(v));
                    return true;
                },
                [&](uint32_t v, double dv, uint32_t j, bool valid) {
                    if (!valid) return;
                    uint32_t u;
                    double w;
                    adj_load(g, j, u, w);
                    const unsigned long long du = D.get(u);
                    if (__dadd_rn(bits2d(du), w) == dv) {
                        atomicMin(&best[v], du);
                        atomicAdd(&cntc[v], 1u);
                        atomicMin(&bslot[v], j);
                    }
                });
            // vertices with several candidates: recount at the minimum
            if (tid == 0) L.qtail = 0;
            __syncthreads();
            for (uint32_t ib = 0; ib < nS; ib += kSsspBlock) {
                const uint32_t i = ib + tid;
                bool multi = false;
                uint32_t v = 0;
                if (i < nS) {
                    v = fscr[i];
                    multi = ld_l2_u32(&cntc[v]) > 1u;
                    if (multi) {
                        atomicExch(&cntc[v], 0u);
                        atomicExch(&bslot[v], 0xFFFFFFFFu);
                    }
                }
                wave_push(multi, v, pnxt, &L.qtail, cap, stats);
            }
            __syncthreads();
            const uint32_t nM = min(L.qtail, cap);
            __syncthreads();
            if (nM > 0) {
                expand_queue(
                    pnxt, nM, g, L,
                    [&](uint32_t v, double& val) {
                        val = bits2d(D.get(v));
                        return true;
                    },
                    [&](uint32_t v, double dv, uint32_t j, bool valid) {
                        if (!valid) return;
                        uint32_t u;
                        double w;
                        adj_load(g, j, u, w);
                        const unsigned long long du = D.get(u);
                        if (__dadd_rn(bits2d(du), w) == dv && du == ld_l2_u64(&best[v])) {
                            atomicAdd(&cntc[v], 1u);
                            atomicMin(&bslot[v], j);
                        }
                    });
            }
            for (uint32_t i = tid; i < nS; i += kSsspBlock) {
                const uint32_t v = fscr[i];
                const uint32_t j = ld_l2_u32(&bslot[v]);
                const uint32_t c = ld_l2_u32(&cntc[v]);
                if (j == 0xFFFFFFFFu) {  // unreachable (cannot happen on a connected graph)
                    atomicAdd(&stats[ST_ERRORS], 1ull);
                    memo[v] = mtag | 0x7FFFFFFFull;
                    par[v] = src;
                } else {
                    memo[v] = mtag | (c > 1 ? 0x80000000ull : 0ull) | (unsigned long long)j;
                    par[v] = adj_col(g, j);
                }
            }
            __syncthreads();
            iter++;
            if (tid == 0) L.qtail = 0;
            __syncthreads();
            for (uint32_t ib = 0; ib < nF; ib += kSsspBlock) {
                const uint32_t i = ib + tid;
                bool p = false;
                uint32_t u = 0;
                if (i < nF) {
                    u = par[pcur[i]];
                    p = (u != src) && ((memo[u] & 0xFFFFFFFF00000000ull) != mtag) &&
                        (atomicExch(&stamp[u], iter) != iter);
                    if (p) { best[u] = kInfBits; cntc[u] = 0; bslot[u] = 0xFFFFFFFFu; }
                }
                wave_push(p, u, pnxt, &L.qtail, cap, stats);
            }
            __syncthreads();
            nF = min(L.qtail, cap);
            uint32_t* t = pcur; pcur = pnxt; pnxt = t;
            __syncthreads();
        }

        { unsigned long long t = wall_clock64(); t_par += t - tk; tk = t; }
        // ---------------- per-target latency / reliability / hops (shd-topology.c:561-671) ----
        double rmin = INFINITY;
        const size_t rowbase = (size_t)s_idx * (size_t)A;
        for (uint32_t k = tid; k < (uint32_t)A; k += kSsspBlock) {
            const uint32_t t = targets[k];
            double lat, rel;
            uint32_t h = 0;
            if (t == src) {
                // path [src]: the self loop (n == 1 branch), no destination loss
                const double sl = g.selfLat[src];
                if (isnan(sl)) {
                    atomicAdd(&stats[ST_ERRORS], 1ull);
                    lat = -1.0;
                    rel = -1.0;
                } else {
                    lat = 0.0 + sl;
                    rel = 1.0;
                    rel *= (1.0 - g.vloss[src]);
                    rel *= (1.0 - g.selfLoss[src]);
                    h = 1;
                }
            } else {
                lat = bits2d(D.get(t));
                bool amb = false, bad = false;
                uint32_t v = t;
                while (v != src) {
                    const unsigned long long m = memo[v];
                    if ((m & 0xFFFFFFFF00000000ull) != mtag || (m & 0x7FFFFFFFull) == 0x7FFFFFFFull) {
                        bad = true;
                        break;
                    }
                    amb |= (m >> 31) & 1ull;
                    if (h < kMaxHops) pbuf[(size_t)h * kSsspBlock + tid] = (uint32_t)(m & 0x7FFFFFFFull);
                    h++;
                    v = par[v];
                    if (h > (uint32_t)V) { bad = true; break; }
                }
                rel = 1.0;
                rel *= (1.0 - g.vloss[src]);
                rel *= (1.0 - g.vloss[t]);
                if (bad) {
                    atomicAdd(&stats[ST_ERRORS], 1ull);
                    lat = -1.0;
                    rel = -1.0;
                } else if (h <= (uint32_t)kMaxHops) {
                    for (int i = (int)h - 1; i >= 0; --i)
                        rel *= (1.0 - g.aloss[pbuf[(size_t)i * kSsspBlock + tid]]);
                } else {
                    atomicAdd(&stats[ST_LONGPATH], 1ull);
                    for (int i = (int)h - 1; i >= 0; --i) {  // edge at depth i from t
                        uint32_t x = t;
                        for (int s = 0; s < i; ++s) x = par[x];
                        rel *= (1.0 - g.aloss[(uint32_t)(memo[x] & 0x7FFFFFFFull)]);
                    }
                }
                if (amb) {
                    atomicAdd(&stats[ST_AMBIGUOUS], 1ull);
                    if (ws.rowflag) ws.rowflag[s_idx] = 1;  // tie replay (topo_replay.hip)
                }
                if (lat == 0.0) lat = 1.0;
            }
            out_lr[rowbase + k] = make_double2(lat, rel);
            out_hops[rowbase + k] = (uint16_t)(h > 65535u ? 65535u : h);
            if (lat >= 0.0) rmin = fmin(rmin, lat);
        }
        // row minimum (feeds the runahead, shd-topology.c:500-511)
        {
            unsigned long long m = d2bits(rmin);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                unsigned long long y = __shfl_xor(m, o, 64);
                m = y < m ? y : m;
            }
            if (tid == 0) L.dmin = kInfBits;
            __syncthreads();
            if ((tid & 63) == 0) atomicMin(&L.dmin, m);
            __syncthreads();
            if (tid == 0) {
                if (out_rowmin) out_rowmin[s_idx] = bits2d(L.dmin);
                atomicMin(&stats[ST_GLOBAL_MIN], L.dmin);
            }
        }
        __syncthreads();
        { unsigned long long t = wall_clock64(); t_tgt += t - tk; tk = t; }
    }
    if (tid == 0) {
        if (nfarscan) atomicAdd(&stats[ST_FARSCAN], nfarscan);
        ctr[0] = iter;
        ctr[2] = mep;
        atomicAdd(&stats[ST_RELAX], relax_local);
        atomicAdd(&stats[ST_T_INIT], t_init);
        atomicAdd(&stats[ST_T_SSSP], t_sssp);
        atomicAdd(&stats[ST_T_PARENT], t_par);
        atomicAdd(&stats[ST_T_TARGET], t_tgt);
        atomicAdd(&stats[ST_T_SPLIT], t_split);
        atomicAdd(&stats[ST_NEAR_IT], n_near);
        atomicAdd(&stats[ST_SPLITS], n_split);
        atomicAdd(&stats[ST_EV0 + 0], ev0);
        atomicAdd(&stats[ST_EV0 + 3], ev3);
        atomicAdd(&stats[ST_EV0 + 4], ev4);
        atomicAdd(&stats[ST_EV0 + 5], ev5);
    }
    if constexpr (EV) {  // per-lane event counts -> one atomic per wave
        for (int k = 0; k < 8; k++) {
            unsigned long long x = ev[k];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if ((tid & 63) == 0 && x) atomicAdd(&stats[ST_EV0 + k], x);
        }
    }
}

// ------------------------------------------------------------------------------------------
// complete graphs: _topology_lookupPath (shd-topology.c:835-873) for every attached pair.
// 34 B of HBM traffic per pair (8 B lat + 8 B loss read, 16 B record + 2 B hops written).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
pair_table_complete_kernel(int A, int64_t row0, int64_t rows, const double* __restrict__ elatAA,
                           const double* __restrict__ elossAA, const double* __restrict__ vlossA,
                           double2* __restrict__ out_lr, uint16_t* __restrict__ out_hops,
                           double* __restrict__ out_rowmin, unsigned long long* __restrict__ stats) {
    const int64_t total = rows * (int64_t)A;
    unsigned long long m = kInfBits;
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = k / A;
        const int64_t c = k - r * A;
        const int64_t i = row0 + r;
        const double el = elatAA[i * A + c];
        double lat, rel;
        if (el < 0.0) {  // no edge between the pair: igraph_get_eid fails (shd-topology.c:857)
            atomicAdd(&stats[ST_ERRORS], 1ull);
            lat = -1.0;
            rel = -1.0;
        } else {
            rel = 1.0;
            rel *= (1.0 - vlossA[i]);
            rel *= (1.0 - vlossA[c]);
            lat = 0.0;
            lat += el;
            rel *= (1.0 - elossAA[i * A + c]);
            unsigned long long b = d2bits(lat);
            m = b < m ? b : m;
        }
        out_lr[k] = make_double2(lat, rel);
        out_hops[k] = 1;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long y = __shfl_xor(m, o, 64);
        m = y < m ? y : m;
    }
    if ((threadIdx.x & 63) == 0 && m != kInfBits) atomicMin(&stats[ST_GLOBAL_MIN], m);
    (void)out_rowmin;
}

// per-row minimum for the complete table (lazy-runahead bookkeeping)
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

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static int grid_for(int64_t n, int block) {
    int64_t g = (n + block - 1) / block;
    if (g > 256 * 16) g = 256 * 16;  // 16 workgroups per CU, grid-stride beyond
    if (g < 1) g = 1;
    return (int)g;
}

SsspLdsPlan sssp_lds_plan(int wg_per_cu, int64_t hub_limit, uint32_t par_hubs, int64_t V) {
    const size_t budget = kSsspMaxLds / (size_t)(wg_per_cu > 1 ? wg_per_cu : 1);
    uint32_t P = par_hubs < kParHubs ? par_hubs : kParHubs;
    // largest H whose layout fits the budget (8 B of distance + 1 bit per hub)
    int64_t H = 0;
    const size_t fixed = lds_layout(0, P).bytes + 8;
    if (budget > fixed) H = (int64_t)((budget - fixed) * 32 / (32 * 8 + 1));
    while (H > 0 && lds_layout((uint32_t)H, P).bytes > budget) H--;
    if (hub_limit >= 0 && hub_limit < H) H = hub_limit;
    if (H > V) H = V;
    if (P > (uint32_t)H) P = (uint32_t)H;
    SsspLdsPlan p;
    p.H = (uint32_t)H;
    p.P = P;
    p.bytes = lds_layout(p.H, p.P).bytes;
    return p;
}

hipError_t launch_sssp_rows(const DevCSR& g, const SlotWs& ws, const uint32_t* d_sources,
                            int nsrc, const uint32_t* d_targets, int A, double delta,
                            const SsspLdsPlan& plan, uint32_t far_cap,
                            uint32_t near_cap, bool events,
                            double2* out_lr,
                            uint16_t* out_hops, double* out_rowmin, unsigned long long* d_stats,
                            hipStream_t stream) {
    int grid = ws.slots < nsrc ? ws.slots : nsrc;
    if (grid < 1) return hipSuccess;
    if ((int64_t)plan.H > g.V || plan.P > plan.H || plan.bytes > kSsspMaxLds ||
        lds_layout(plan.H, plan.P).bytes != plan.bytes)
        return hipErrorInvalidValue;
    const uint32_t hubs = plan.H, par_hubs = plan.P;
    const size_t lds = plan.bytes;
    {  // per device (multi-GPU builds launch on several): set before every launch
        for (const void* k : {(const void*)sssp_rows_kernel<false>,
                              (const void*)sssp_rows_kernel<true>}) {
            hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)kSsspMaxLds);
            if (e != hipSuccess) return e;
        }
    }
    hipLaunchKernelGGL(events ? sssp_rows_kernel<true> : sssp_rows_kernel<false>, dim3(grid),
                       dim3(kSsspBlock), lds, stream, g, ws,
                       d_sources, nsrc, d_targets, A, delta, hubs, par_hubs, far_cap, near_cap,
                       out_lr,
                       out_hops,
                       out_rowmin, d_stats);
    return hipGetLastError();
}

hipError_t launch_pair_table_complete(int A, int64_t row0, int64_t rows, const double* elatAA,
                                      const double* elossAA, const double* vlossA, double2* out_lr,
                                      uint16_t* out_hops, double* out_rowmin,
                                      unsigned long long* d_stats, hipStream_t stream) {
    if (rows <= 0 || A <= 0) return hipSuccess;
    hipLaunchKernelGGL(pair_table_complete_kernel, dim3(grid_for(rows * A, 256)), dim3(256), 0,
                       stream, A, row0, rows, elatAA, elossAA, vlossA, out_lr, out_hops,
                       out_rowmin, d_stats);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !out_rowmin) return e;
    hipLaunchKernelGGL(row_min_kernel, dim3((unsigned)rows), dim3(256), 0, stream, rows,
                       (int64_t)A, out_lr, out_rowmin);
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

int sssp_max_blocks_per_cu(int wg_per_cu) {
    const SsspLdsPlan p = sssp_lds_plan(wg_per_cu, -1, kParHubs, INT64_MAX);
    int nb = 0;
    if (hipFuncSetAttribute((const void*)sssp_rows_kernel<false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSsspMaxLds) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sssp_rows_kernel<false>, kSsspBlock,
                                                     p.bytes) != hipSuccess)
        return 1;
    return nb < 1 ? 1 : nb;
}

}  // namespace shdtopo
