// topo_sssp_batch.hip -- batched multi-source SSSP for gfx950: one persistent workgroup settles
// K sources at once (K = 8: the K distances of a vertex are one 64-B line).
//
// Replaces igraph_get_shortest_paths_dijkstra + the per-target helper
// (src/topology/shd-topology.c:561-833): same distances (bit-exact: every latency add is one IEEE
// add and any label-correcting order reaches the same monotone-rounding fixpoint), same parents
// (the argmin d[u] rule of SURVEY.md A.3), same per-target epilogue.
//
// Why batch.  The single-source kernel is bound by random 64-B DRAM requests: every relaxation of
// a tail vertex reads (and may atomically lower) one 8-B distance word, i.e. a whole line.  On a
// power-law Internet topology almost every shortest path runs through the hub core, so
// d_s(v) ~= d_s(h0) + d(h0, v) for the top hub h0: shifted by pi(s) = d(h0, s), the distances of
// different sources to the same vertex fall into the same or adjacent delta-buckets (measured on
// C4: 8 random sources, delta = 3 ms, 1.84 distinct buckets per vertex).  Lock-step buckets over
// the shifted keys therefore expand a vertex ONCE for all sources that reach it in the current
// bucket: the adjacency row is read once, and each relaxation reads the target's K distances as
// one line.  The (edge, source) pairs of an edge sit in adjacent lanes.
//
// Per-source correctness is untouched by the shift: source j's bucket of a distance d is
// floor((d + sh_j) / delta) with sh_j = C - pi(s_j) >= 0, a monotone function of d, and source j's
// buckets are settled in increasing order -- lock-step only interleaves independent sources.
//
// Near-phase bookkeeping per vertex: a K-bit mask of the sources that must expand it in the next
// iteration (double buffered by iteration parity; hubs' masks in LDS).  A vertex enters the next
// near queue when its mask goes from 0 to non-zero, so the queue is deduplicated (<= V entries)
// and an expansion serves every source of the mask.
//
// Far improvements are not queued at all: they only lower L.fminb, the smallest pending bucket.
// Each bucket starts with one streaming sweep over the batch's [V][K] rows (16-B loads, 64 MB at
// K = 8) that classifies every (vertex, source) by its current bucket and builds the bucket's
// near queue and masks.  With wide buckets (delta ~ 0.2 x mean edge latency, ~25 buckets per
// batch on C4) the sweeps are cheaper than per-(vertex, source) queue entries, which cost random
// reads and atomics to merge (measured: DESIGN.md 4).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <type_traits>

#include "topo_dev_common.h"

namespace shdtopo {

namespace {

using namespace dev;

// Tuning constants (A/B measured): phase-B rounds whose loads are in flight together
// (2 < 3 < 4 by 1-4 %, 8 spills), phase-A edges per lane, queue vertices per expansion chunk.
// Round 6 removed the measured-slower variants that were compiled in behind SHD_* switches (the
// help board, the pending-vertex sweep list, speculative hub buckets, the phase-B target skip,
// node-major walks, temporal stores of the reset and the table, the mask read + store pair); their
// A/B numbers stay in DESIGN.md 4 and the code in git history.
constexpr int kBatchRB = 2;
constexpr int kBatchU = 2;
constexpr int kBChunk = 512;  // (<= kSsspBlock)
#ifndef SHD_BATCH_WRCOUNT
#define SHD_BATCH_WRCOUNT 0  // profiling build: 64-B lines written per category (ST_WL0)
#endif
#ifndef SHD_BATCH_TIME
#define SHD_BATCH_TIME 0  // profiling build: per-wave time of the near iterations' parts
#endif
#if SHD_BATCH_TIME
#define BT_TICK(i) do { const unsigned long long t_ = wall_clock64(); \
    if ((threadIdx.x & 63) == 0) atomicAdd(&L.bt[(WAVE ? 0 : 3) + (i)], t_ - bt_last); bt_last = t_; } while (0)
#else
#define BT_TICK(i) do { } while (0)
#endif
constexpr uint32_t kNoBucket = 0xFFFFFFFFu;
constexpr size_t kBMaxLds = 160 * 1024 / kBatchWgPerCu;  // a CU's LDS over its workgroups

template <int K>
struct MaskOps {
    static_assert(K == 2 || K == 4 || K == 8 || K == 16, "batch width");
    using M = typename std::conditional<(K <= 8), uint8_t, uint16_t>::type;
    static constexpr int kBits = 8 * (int)sizeof(M);
    static constexpr int kPer = 32 / kBits;
    static constexpr uint32_t kFull = (1u << K) - 1u;
    // returning OR of `bits` into v's mask (LDS or HBM word); returns v's previous mask
    __device__ static __forceinline__ uint32_t set(M* m, uint32_t v, uint32_t bits) {
        uint32_t* w = reinterpret_cast<uint32_t*>(m) + v / kPer;
        const uint32_t s = (v % kPer) * kBits;
        return (atomicOr(w, bits << s) >> s) & kFull;
    }
    // atomic read-and-clear of v's mask (hub masks are OR-ed by other waves while they are read)
    __device__ static __forceinline__ uint32_t take(M* m, uint32_t v) {
        uint32_t* w = reinterpret_cast<uint32_t*>(m) + v / kPer;
        const uint32_t s = (v % kPer) * kBits;
        return (atomicAnd(w, ~(kFull << s)) >> s) & kFull;
    }
    // HBM mask read that bypasses L1 (the words are written by atomics of other waves)
    __device__ static __forceinline__ uint32_t get_l2(const M* m, uint32_t v) {
        const uint32_t w = ld_l2_u32(reinterpret_cast<const uint32_t*>(m) + v / kPer);
        return (w >> ((v % kPer) * kBits)) & kFull;
    }
};

template <int K>
struct LdsB {
    uint32_t off[kBChunk + 4];
    uint32_t rs[kBChunk];
    uint32_t vx[kBChunk];
    uint32_t msk[kBChunk];
    double val[kBChunk * K];  // the chunk's source distances, [vertex][source]
    double sh[K];             // per-source bucket shift sh_j = C - pi(s_j)
    double dh0[K];            // per-source d_j(h0) (landmark filter; refreshed per chunk)
    double invd;              // 1 / delta
    uint32_t wave[kSsspBlock / 64];
    uint32_t qtail;
    uint32_t qhead;    // next queue entry taken by a wave (tail iterations, wave sub-chunks)
    uint32_t htail;    // hubs waiting in the deferred hub list
    uint32_t idx;      // batch taken by this workgroup
    uint32_t src[K];   // the batch's source vertices
    uint32_t fover;    // a (deduplicated, V-entry) queue overflowed: cannot happen, reported
    uint32_t fminb;    // smallest bucket of the pending (vertex, source) pairs past cb
    unsigned long long rmin[K];  // per-source row minimum of the batch's table rows
    unsigned long long cnt[4];  // source-relaxations, sweep entries, edges, chunk-setup ticks
    unsigned long long pt[5];   // parent-pass phase ticks (diagnostic)
    unsigned long long dg[4];   // diagnostic: hub edges, hub source-relaxations, first-iteration
                                // edges, first-iteration source-relaxations
    unsigned long long touched; // tail lines reset (touched by the slot's previous batches)
    unsigned long long wk[5];   // parent pass: walk steps; resolved by the h0-tree guess, a
                                // tail's improver, a hub's improver; pairs sent to row scans
    unsigned long long bt[8];   // SHD_BATCH_TIME builds: wave ticks of tail / hub iterations in
                                // chunk loads, phase A, phase B; phase-B rounds, active lanes
    unsigned long long sw[4];   // SHD_BATCH_TIME builds (ST_SW0): phase-B rounds with a tail
                                // target, tail-target pairs, hub-target pairs, (unused)
    // per-workgroup counters and phase ticks, kept here by thread 0 rather than in (uniform)
    // registers: near iterations, sweeps, expansions, parent-pass pairs; ticks of init, SSSP,
    // parents, targets, sweeps; the last tick
    unsigned long long ev[4];
    unsigned long long tm[5];
    unsigned long long tk;
    unsigned long long wl[16];  // SHD_BATCH_WRCOUNT builds: 64-B lines stored / atomically
                                // written per category (WL_*), then read per category (RL_*)
    unsigned long long rl[16];
    // jobs (a level's walks, the epilogue): the cursor of the current job's items
    uint32_t jcur;
    uint32_t rsb;  // parent pass: the current row-scan chunk's first R entry
};

// Write categories of SHD_BATCH_WRCOUNT builds (ShdStats.write_lines): each store / atomic
// wave-instruction adds the 64-B lines its active lanes touch (a lane whose line equals its
// predecessor's counts once, so coalesced runs count their lines and scattered lanes one each).
enum {
    WL_RELAX_MIN,    // relaxation: returning atomicMin of a tail distance
    WL_RELAX_TIE,    //   tie tag stores
    WL_RELAX_HINT,   //   improver hint stores
    WL_RELAX_PEND,   //   (unused: pending and touched bits share one atomic, WL_RELAX_TOUCH)
    WL_RELAX_TOUCH,  //   first-reach atomics (touched + pending bits)
    WL_RELAX_MASK,   //   near-mask atomics (HBM)
    WL_MASK_ST,      // mask stores (chunk loads clear, sweeps set)
    WL_PEND_ST,      // pending words (batch init, sweep rewrites)
    WL_RESET,        // touched distance lines reset to +inf
    WL_TOUCH_CLR,    // touched words cleared
    WL_PREC,         // pair records (walk puts, tags, hint puts, row-scan results)
    WL_PSCR,         // parent-pass scratch (row-scan records, row-scan vertex masks)
    WL_OUT,          // table rows, hops, row minima, row flags
    WL_HUB,          // hub rows copied to their dist rows, hub parent hints
    WL_QUEUE,        // queue / list appends (near queues, hub lists, pair lists)
    WL_OTHER         // path buffer spill to HBM, source init
};
// Read categories of SHD_BATCH_WRCOUNT builds (ShdStats.read_lines), counted like the writes.
enum {
    RL_RELAX_PRE,  // phase B pre-check of the target's distance line
    RL_PHASE_A,    // phase A adjacency records (kappa-sorted copy)
    RL_CHUNK,      // chunk / sub-chunk loads: queue entries, masks, row bounds, probes, distances
    RL_SWEEP,      // sweeps: bitmap words, kappa0, distance lines
    RL_WALK,       // parent walks: start pairs, tag words, tree records, distances
    RL_EPI,        // epilogue: targets, vertex arrays, distances, pair records
    RL_RESET,      // reset: bitmap words
    RL_OTHER       // hint pass and row scans
};
template <int K>
__device__ __forceinline__ void rl_count(LdsB<K>& L, int cat, bool act, const void* a) {
#if SHD_BATCH_WRCOUNT
    const unsigned long long line = (unsigned long long)a >> 6;
    const unsigned long long am = __ballot(act);
    if (!am) return;
    const int lane = (int)(threadIdx.x & 63u);
    const unsigned long long prev = __shfl_up(line, 1, 64);
    const bool dup = lane > 0 && ((am >> (lane - 1)) & 1ull) && prev == line;
    const unsigned long long nm = __ballot(act && !dup);
    if (lane == __ffsll((long long)am) - 1) atomicAdd(&L.rl[cat], (unsigned long long)__popcll(nm));
#else
    (void)L; (void)cat; (void)act; (void)a;
#endif
}
template <int K>
__device__ __forceinline__ void wl_count(LdsB<K>& L, int cat, bool act, const void* a) {
#if SHD_BATCH_WRCOUNT
    const unsigned long long line = (unsigned long long)a >> 6;
    const unsigned long long am = __ballot(act);
    if (!am) return;
    const int lane = (int)(threadIdx.x & 63u);
    const unsigned long long prev = __shfl_up(line, 1, 64);
    const bool dup = lane > 0 && ((am >> (lane - 1)) & 1ull) && prev == line;
    const unsigned long long nm = __ballot(act && !dup);
    if (lane == __ffsll((long long)am) - 1) atomicAdd(&L.wl[cat], (unsigned long long)__popcll(nm));
#else
    (void)L; (void)cat; (void)act; (void)a;
#endif
}

// wave_push_t (topo_dev_common.h) that also counts its queue stores (SHD_BATCH_WRCOUNT)
template <int K>
__device__ __forceinline__ void wpush(LdsB<K>& L, bool pred, uint32_t val, uint32_t* q,
                                      uint32_t* lds_tail, uint32_t cap, uint32_t* lds_over,
                                      uint32_t code) {
    unsigned long long m = __ballot(pred);
    if (m == 0ull) return;
    const int lane = (int)(threadIdx.x & 63u);
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(lds_tail, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    wl_count(L, WL_QUEUE, pred && pos < cap, q + pos);
    if (pred) {
        if (pos < cap) q[pos] = val;
        else atomicOr(lds_over, code);
    }
}

// Dynamic LDS after the control block: the hubs' (deferred) source masks, parent-tie bits of the
// first P hubs (P*K bits), "expanded at its current value" bits of every (hub, source), then the
// hub distances hd[H][K].
struct BLayout {
    size_t hdef, tb, xb, hd, bytes;
};
template <int K>
__host__ __device__ inline BLayout blayout(uint32_t H, uint32_t P) {
    using M = typename MaskOps<K>::M;
    BLayout l;
    const size_t ctrl = (sizeof(LdsB<K>) + 15) / 16 * 16;
    const size_t mb = ((size_t)H * sizeof(M) + 15) / 16 * 16;
    l.hdef = ctrl;
    l.tb = ctrl + mb;
    const size_t tbw = ((size_t)P * K + 31) / 32;
    l.xb = l.tb + 4 * tbw;
    const size_t xbw = ((size_t)H * K + 31) / 32;
    l.hd = (l.xb + 4 * xbw + 15) / 16 * 16;
    l.bytes = l.hd + 8 * (size_t)H * K;
    return l;
}

__device__ __forceinline__ uint32_t bkt(double d, double sh, double inv_delta) {
    return bucket_of(__dadd_rn(d, sh), inv_delta);
}

template <int K>
struct BView {
    using M = typename MaskOps<K>::M;
    unsigned long long* hd;    // LDS [H][K]
    unsigned long long* dist;  // HBM [V][K] (rows < H unused while the batch runs)
    uint32_t* tb;              // LDS parent-tie bits of (hub < P, source)
    uint32_t* xb;              // LDS: (hub, source) expanded at its current distance
    uint32_t* hpar;            // HBM [P][K]: vertex whose relaxation last lowered hub v for j
    // HBM, 2 bits per vertex (16 vertices per word): bit 2i a pair of vertex i pending past cb,
    // bit 2i + 1 the batch lowered its line from +inf (touched: reset at the batch's end).  A
    // pending vertex is always touched, so one atomic sets both and the reset clears both.
    uint32_t* pt;
    uint32_t* tpar;            // HBM [V][K] pair records: word 0 = vertex whose relaxation last
                               // lowered the tail pair (the parent field before
                               // the parent pass), word 1 = tag word (ties: kTagTie)
    uint32_t H, P;
    __device__ __forceinline__ unsigned long long get(uint32_t v, uint32_t j) const {
        return v < H ? hd[(size_t)v * K + j] : ld_l2_u64(&dist[(size_t)v * K + j]);
    }
};

struct BBuckets {
    double inv_delta;
    uint32_t cb;       // the bucket being settled
    uint32_t tie_tag;  // the batch's tag | kTagTie (pair records of tied tail pairs)
};

// Pair record tag word (word 1 of the 16-B record): the batch tag ep (30 bits, 1..kTagMask) |
// kTagClaim once the parent pass resolved or claimed the pair | kTagTie when a relaxation of this
// batch tied the pair's value (set during the SSSP, kept on a claim).  Tags of other batches match
// nothing, so no per-batch clearing is needed.
constexpr uint32_t kTagMask = 0x3FFFFFFFu;
constexpr uint32_t kTagClaim = 0x40000000u;
constexpr uint32_t kTagTie = 0x80000000u;
__device__ __forceinline__ bool tag_claimed(uint32_t w, uint32_t ep) {
    return (w & ~kTagTie) == (ep | kTagClaim);
}
__device__ __forceinline__ bool tag_tied(uint32_t w, uint32_t ep) {
    return (w & kTagTie) && (w & kTagMask) == ep;
}

// End of the kappa-sorted row prefix that can pass threshold T: the first probe position
// (0, 1, 3, 7[, 15, 31, 63, 127]) whose kappa exceeds T (an upper bound: the edges before it are
// filtered per source in phase A), else a binary search past the last probe (long rows only).
__device__ __forceinline__ uint32_t kappa_cut(const DevCSR& g, float4 ks0, float4 ks1, double T,
                                              uint32_t r0, uint32_t deg) {
    if ((double)ks0.x > T) return 0;
    if ((double)ks0.y > T) return 1;
    if ((double)ks0.z > T) return 3;
    if ((double)ks0.w > T) return 7;
    if (kKProbes > 4) {
        if ((double)ks1.x > T) return 15;
        if ((double)ks1.y > T) return 31;
        if ((double)ks1.z > T) return 63;
        if ((double)ks1.w > T) return 127;
    }
    uint32_t lo = kKProbes > 4 ? 128u : 8u, hi = deg;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((double)g.kap[r0 + mid] > T) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// One chunk of a near queue: take each vertex's source mask (clearing it), its row bounds and
// its K distances (K lanes per vertex read its line once) into LDS; a block scan of the degrees
// flattens the chunk's edges.  Returns the chunk's edge count (uniform); ends with a barrier.
// CUT (relaxation): rows are the kappa-sorted copy and only the prefix that can pass the
// landmark filter for some source of the mask is taken (kappa <= max_j d_j(h0) - d_j(v) plus a
// margin wider than the filter's); its K distances are read by the vertex's thread with the row
// bounds.  Without CUT (parent pass) whole rows of the id-sorted adjacency.
template <int K, bool CUT = false, bool DIR = false>
__device__ __forceinline__ uint32_t load_chunk(const uint32_t* Q, uint32_t cnt, const DevCSR& g,
                                               LdsB<K>& L, const BView<K>& D,
                                               typename MaskOps<K>::M* mcur,
                                               typename MaskOps<K>::M* hcur, bool stats = true,
                                               uint32_t spec_to = 0u) {
    using MO = MaskOps<K>;
    const uint32_t tid = threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    uint32_t deg = 0;
    unsigned long long act = 0;
    if (tid < cnt) {
        const uint32_t v = Q[tid];
        uint32_t m;
        if (v < D.H) {
            m = MO::take(hcur, v);
            if (spec_to) {
                // speculative co-expansion: the row also serves every source whose tentative
                // distance lies in the next buckets (<= spec_to) and has not been expanded yet.
                // Exact either way: a later improvement clears the source's x bit and queues the
                // hub again; a final one is never expanded twice (the sweep skips x bits).
                const uint32_t xw = D.xb[(v * K) >> 5] >> ((v * K) & 31);
                for (int jj = 0; jj < K; jj++) {
                    if (((m >> jj) & 1u) || ((xw >> jj) & 1u)) continue;
                    const unsigned long long d = D.hd[(size_t)v * K + jj];
                    if (d != kInfBits && bkt(bits2d(d), L.sh[jj], L.invd) <= spec_to) m |= 1u << jj;
                }
                if (m) atomicOr(&D.xb[(v * K) >> 5], m << ((v * K) & 31));
            }
        } else {
            wl_count(L, WL_MASK_ST, true, mcur + v);
            m = MO::take(mcur, v);  // read-and-clear: one returning atomic
        }
        // relaxation: the out-rows (kappa copy); parent pass: the rows of candidate parents (the
        // in-rows of a directed topology)
        const uint32_t* rp = (CUT || !DIR) ? g.rowptr : g.rowptr_in;
        const uint32_t r0 = rp[v], r1 = rp[v + 1];
        deg = m ? r1 - r0 : 0u;
        if (CUT && deg) {
            const float4 ks0 = g.ksum[kKProbes / 4 * (size_t)v];
            const float4 ks1 = kKProbes > 4 ? g.ksum[kKProbes / 4 * (size_t)v + 1] : ks0;
            double dv[K];
            if (v < D.H) {
#pragma unroll
                for (int jj = 0; jj < K; jj++) dv[jj] = bits2d(D.hd[(size_t)v * K + jj]);
            } else {
                typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                const u64x2* p = reinterpret_cast<const u64x2*>(D.dist + (size_t)v * K);
#pragma unroll
                for (int h = 0; h < K / 2; h++) {
                    const u64x2 x = __builtin_nontemporal_load(p + h);
                    dv[2 * h] = bits2d(x.x);
                    dv[2 * h + 1] = bits2d(x.y);
                }
            }
            // threshold: kappa <= d_j(h0) - d_j(v) + 1e-5 (d_j(h0) + d_j(v) + piMax) for some j
            // of the mask (the filter's own margin is 1e-6 relative); +inf keeps the whole row
            double T = -INFINITY;
#pragma unroll
            for (int jj = 0; jj < K; jj++) {
                if (!((m >> jj) & 1u)) continue;
                L.val[tid * K + jj] = dv[jj];
                const double h = bits2d(D.get(0u, (uint32_t)jj));
                const double t = (h - dv[jj]) + 1e-5 * (h + dv[jj] + g.piMax) + 1e-9;
                T = t > T ? t : T;
            }
            const uint32_t c = kappa_cut(g, ks0, ks1, T, r0, deg);
            deg = c < deg ? c : deg;
        }
        act = (unsigned long long)deg * (unsigned long long)__popc(m);
        L.rs[tid] = r0;
        L.vx[tid] = v;
        L.msk[tid] = m;
        if (stats && v < D.H && deg) {
            atomicAdd(&L.dg[0], (unsigned long long)deg);
            atomicAdd(&L.dg[1], act);
        }
    }
    uint32_t total;
    const uint32_t off = block_excl_scan<kSsspBlock>(deg, L.wave, &total);
    if (tid < cnt) L.off[tid] = off;
    if (tid == 0) L.off[cnt] = total;
    act = wave_sum_u64(act);
    if (stats && (tid & 63) == 0 && act) atomicAdd(&L.cnt[0], act);
    if (!CUT) {
        for (uint32_t i = tid; i < cnt * K; i += kSsspBlock) {
            const uint32_t vi = i / K, jj = i % K;
            if ((L.msk[vi] >> jj) & 1u) L.val[i] = bits2d(D.get(L.vx[vi], jj));
        }
    }
    if (tid < (uint32_t)K) L.dh0[tid] = bits2d(D.get(0u, tid));
    __syncthreads();
    if (stats && tid == 0) {
        L.cnt[2] += total;
        L.cnt[3] += wall_clock64() - t0;
    }
    return total;
}

// Can vertex v at distance d (source j, d_j(h0) = h) have an edge that passes the landmark
// filter?  Only if kappa0(v) (its smallest kappa, f32 rounded down) lies under the CUT threshold of
// load_chunk; h may be stale (larger), which only widens the test.
// the record's pi(col) (rounded up) and the target's kappa0 (rounded down), kKapInRec layout
__device__ __forceinline__ double rec_pi(uint32_t p) {
    if (kKapInRec) return (double)(float)__builtin_bit_cast(_Float16, (unsigned short)(p >> 16));
    return (double)__uint_as_float(p);
}
__device__ __forceinline__ float rec_kap0(uint32_t p) {
    return (float)__builtin_bit_cast(_Float16, (unsigned short)(p & 0xFFFFu));
}

__device__ __forceinline__ bool kappa_useful(float k0, double h, double d, double pimax) {
    return (double)k0 <= (h - d) + 1e-5 * (h + d + pimax) + 1e-9;
}

// Edge index e of the chunk -> its vertex slot in the chunk (binary search over L.off).
template <int K>
__device__ __forceinline__ int chunk_slot(const LdsB<K>& L, uint32_t cnt, uint32_t e) {
    int lo = 0, hi = (int)cnt - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (L.off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Wave-wide exclusive prefix sum (no barrier); *total = the wave's sum.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(v, o, 64);
        if (lane >= (uint32_t)o) v += y;
    }
    *total = __shfl(v, 63, 64);
    return v - x;
}

// Slot of edge e in a (wave's) chunk slice: binary search over its cnt offsets.
__device__ __forceinline__ uint32_t slice_slot(const uint32_t* off, uint32_t cnt, uint32_t e) {
    uint32_t lo = 0, hi = cnt - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Wave sub-chunk of a TAIL queue (tail iterations): like load_chunk<K, true>, but one wave loads
// up to kBSub vertices into its own slice [wb, wb + kBSub) of the chunk arrays and flattens
// their cut rows with a wave scan, so the waves of a workgroup run their sub-chunks without
// barriers.  Returns the slice's edge count (wave-uniform).
constexpr uint32_t kBSub = kBChunk / (kSsspBlock / 64);
template <int K>
__device__ __forceinline__ uint32_t load_sub(uint32_t qv, uint32_t cnt, uint32_t wb,
                                             const DevCSR& g, LdsB<K>& L, const BView<K>& D,
                                             typename MaskOps<K>::M* mcur) {
    using MO = MaskOps<K>;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t deg = 0;
    unsigned long long act = 0;
    if (lane < K) L.dh0[lane] = bits2d(D.get(0u, lane));  // any value read is a valid bound
    if (lane < cnt) {
        const uint32_t v = qv;  // this lane's queue entry (loaded by the caller)
        // every load of the vertex in one round trip: its mask (a queued vertex's is almost
        // never empty), row bounds, kappa probes and K distances
        wl_count(L, WL_MASK_ST, true, mcur + v);
        const uint32_t m = MO::take(mcur, v);  // read-and-clear: one returning atomic
        rl_count(L, RL_CHUNK, true, mcur + v);
        rl_count(L, RL_CHUNK, true, g.rowptr + v);
        rl_count(L, RL_CHUNK, true, g.ksum + kKProbes / 4 * (size_t)v);
        rl_count(L, RL_CHUNK, true, D.dist + (size_t)v * K);
        const uint32_t r0 = g.rowptr[v], r1 = g.rowptr[v + 1];
        const float4 ks0 = g.ksum[kKProbes / 4 * (size_t)v];
        const float4 ks1 = kKProbes > 4 ? g.ksum[kKProbes / 4 * (size_t)v + 1] : ks0;
        double dv[K];
        {
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            const u64x2* p = reinterpret_cast<const u64x2*>(D.dist + (size_t)v * K);
#pragma unroll
            for (int h = 0; h < K / 2; h++) {
                const u64x2 x = __builtin_nontemporal_load(p + h);
                dv[2 * h] = bits2d(x.x);
                dv[2 * h + 1] = bits2d(x.y);
            }
        }
        deg = m ? r1 - r0 : 0u;
        if (deg) {
            double T = -INFINITY;
#pragma unroll
            for (int jj = 0; jj < K; jj++) {
                if (!((m >> jj) & 1u)) continue;
                L.val[(wb + lane) * K + jj] = dv[jj];
                const double h = bits2d(D.get(0u, (uint32_t)jj));
                const double t = (h - dv[jj]) + 1e-5 * (h + dv[jj] + g.piMax) + 1e-9;
                T = t > T ? t : T;
            }
            const uint32_t c = kappa_cut(g, ks0, ks1, T, r0, deg);
            deg = c < deg ? c : deg;
        }
        act = (unsigned long long)deg * (unsigned long long)__popc(m);
        L.rs[wb + lane] = r0;
        L.vx[wb + lane] = v;
        L.msk[wb + lane] = m;
    }
    uint32_t total;
    const uint32_t off = wave_excl_scan(deg, &total);
    if (lane < cnt) L.off[wb + lane] = off;
    act = wave_sum_u64(act);
    if (lane == 0) {
        if (act) atomicAdd(&L.cnt[0], act);
        atomicAdd(&L.cnt[2], (unsigned long long)total);
    }
    // the slice's LDS writes are read by other lanes of this wave only
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    return total;
}

// Transposed near iteration: phase A takes one edge per lane (UA per lane in flight: row search
// + 16-B record load done once per edge, not once per source) and applies the landmark filter
// per (edge, source); phase B spreads the surviving (edge, source) pairs over the lanes, 64 per
// round, the pairs of one edge in adjacent lanes: their pre-check loads and atomics hit ONE 64-B
// line per edge in one instruction (coalesced: one DRAM request instead of up to K), and the
// edge's queue bookkeeping is done once by its first lane.  (Edge rounds -- K lanes per edge,
// lane j = source j -- left 39 % of the lanes idle: 38.7 k rounds per source against 25.0 k;
// full C4 table 401 -> 398 ms, 1,250 rows 88.5 -> 84.4 ms.)
// Hubs are deferred: a hub improved into bucket cb sets its bit in hdef (one mask per hub, no
// parity) and joins the hub list hq once; the kernel expands the list only when the tail queue
// is empty, so one hub expansion serves every source that reached it meanwhile (hub rows are
// 41 % of the expanded edges; expanded at once they serve 2.3 sources each).
template <int K, int UA, bool WAVE = false>
__device__ __forceinline__ void relax_batch_t(const uint32_t* Q, uint32_t nq, const DevCSR& g,
                                              LdsB<K>& L, const BView<K>& D,
                                              typename MaskOps<K>::M* mcur,
                                              typename MaskOps<K>::M* hdef,
                                              typename MaskOps<K>::M* mnxt, uint32_t* qout,
                                              uint32_t qcap, uint32_t* hq, const BBuckets& B) {
    using MO = MaskOps<K>;
    static_assert(64 % K == 0, "a wave holds whole edge groups");
    static_assert(UA >= 1 && (UA & (UA - 1)) == 0, "the phase-B edge search halves UA * 64");
    constexpr int RB = kBatchRB;     // phase-B rounds whose loads are in flight together
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    const uint32_t wv = tid >> 6;
    // WAVE (tail iterations): each wave takes kBSub-vertex sub-chunks of the queue from an LDS
    // counter into its own slice of the chunk arrays; no barrier until the iteration ends.
    // Otherwise (hub iterations: long rows) block-wide 512-vertex chunks.
    const uint32_t wb = WAVE ? wv * kBSub : 0u;
    // WAVE: the next sub-chunk is taken and its queue entries loaded before this one is
    // expanded (one global round trip less on each sub-chunk's dependent chain)
    uint32_t nb0 = 0, nqv = 0;
#if SHD_BATCH_TIME
    unsigned long long bt_last = wall_clock64();
#endif
    if (WAVE) {
        if (lane == 0) nb0 = atomicAdd(&L.qhead, kBSub);
        nb0 = __shfl(nb0, 0, 64);
        rl_count(L, RL_CHUNK, nb0 + lane < nq, Q + nb0 + lane);
        nqv = nb0 + lane < nq ? Q[nb0 + lane] : 0u;
    }
    for (uint32_t base = 0;; base += kBChunk) {
        uint32_t cnt, total;
        if (WAVE) {
            const uint32_t b0 = nb0, qv = nqv;
            if (b0 >= nq) break;
            cnt = min(kBSub, nq - b0);
            if (lane == 0) nb0 = atomicAdd(&L.qhead, kBSub);
            nb0 = __shfl(nb0, 0, 64);
            rl_count(L, RL_CHUNK, nb0 + lane < nq, Q + nb0 + lane);
            nqv = nb0 + lane < nq ? Q[nb0 + lane] : 0u;
            total = load_sub<K>(qv, cnt, wb, g, L, D, mcur);
        } else {
            if (base >= nq) break;
            cnt = min((uint32_t)kBChunk, nq - base);
            total = load_chunk<K, true>(Q + base, cnt, g, L, D, mcur, hdef, true,
                                        B.cb);
        }
        BT_TICK(0);
        constexpr uint32_t kStep = WAVE ? 64u : (uint32_t)kSsspBlock;  // lanes per phase-A slot
        for (uint32_t eb = 0; eb < total; eb += kStep * UA) {
            // phase A: edge e = eb + a * kStep (+ wv * 64 block-wide) + lane
            uint32_t an[UA], amk[UA], alo[UA], awl[UA], awh[UA], apb[UA];
#pragma unroll
            for (int a = 0; a < UA; a++) {
                const uint32_t e = eb + (uint32_t)a * kStep + (WAVE ? 0u : wv * 64) + lane;
                const bool valid = e < total;
                const int lo = !valid ? 0
                               : WAVE ? (int)(wb + slice_slot(L.off + wb, cnt, e))
                                      : chunk_slot<K>(L, cnt, e);
                const uint32_t jr = valid ? L.rs[lo] + (e - L.off[lo]) : 0u;
                rl_count(L, RL_PHASE_A, valid, g.adjk + kAdjWords * jr);
                const AdjRec r = *reinterpret_cast<const AdjRec*>(g.adjk + kAdjWords * jr);
                an[a] = r.a;
                apb[a] = r.p;
                awl[a] = r.b;
                awh[a] = r.c;
                amk[a] = valid ? L.msk[lo] : 0u;
                alo[a] = (uint32_t)lo;
            }
            // Landmark filter, per (edge, source) of the lane's edges: the walk s_j -> h0 -> n
            // gives d_j(n) <= d_j(h0) + pi(n) (up to rounding, far inside the 1e-6 margin;
            // pi(n) is stored rounded up, d_j(h0) may be stale, i.e. larger), so a candidate
            // above the bound can neither improve n's final distance nor tie it and the source
            // is dropped from the edge (91 % of the tail relaxations on C4).  Every relaxation
            // that sets or ties a final value is still performed: distances, parent hints and
            // tie bits are unchanged.
            // The target skip is decided here too, per (edge, source): a tail vertex that is no
            // table target and would expand nothing at this candidate (kappa0 above the landmark
            // threshold, the test that keeps it out of the near queue) needs no distance at all --
            // only targets and the vertices of their parent chains are read after the SSSP, and a
            // chain vertex is expanded at its final distance (its chain edge passes the filter),
            // so every relaxation that sets or ties its final value passes this test (a larger,
            // stale d_j(h0) only widens it).  A dropped pair takes no phase-B lane (C4: 21 % of
            // the pairs).
#pragma unroll
            for (int a = 0; a < UA; a++) {
                uint32_t mk = amk[a];
                const double w = __hiloint2double((int)awh[a], (int)awl[a]);
                const double pv = rec_pi(apb[a]);
                const bool skippable = kKapInRec && g.tflags &&
                                       (an[a] & 0x3FFFFFFFu) >= D.H && !((an[a] >> 30) & 1u);
                const float kz0 = rec_kap0(apb[a]);
                while (mk) {
                    const uint32_t jj = (uint32_t)__ffs(mk) - 1u;
                    mk &= mk - 1u;
                    const double ad = __dadd_rn(L.val[alo[a] * K + jj], w);
                    const double bnd = __dmul_rn(__dadd_rn(L.dh0[jj], pv), 1.000001);
                    if (ad > bnd || (skippable && !kappa_useful(kz0, L.dh0[jj], ad, g.piMax)))
                        amk[a] &= ~(1u << jj);
                }
            }
            // Pair compaction: the wave's surviving (edge, source) pairs, in edge order (edge
            // E = a * 64 + lane), 64 per phase-B round; lane l of round r takes pair r * 64 + l:
            // its edge is the last E whose exclusive pair offset is <= the pair's index (binary
            // search over the offsets by shuffles), its source the matching set bit of the
            // edge's mask.  The pairs of one edge sit in adjacent lanes: their loads and atomics
            // on the target's 64-B line of K distances still go out as one request.
            // Two classes of pairs, numbered apart: pairs into tail vertices (HBM line: pre-check
            // load, returning atomicMin) fill the first rounds, pairs into LDS hubs the rest.  A
            // hub round then issues no HBM load or returning atomic at all (LDS atomics and
            // fire-and-forget stores only), instead of waiting on the tail pairs it was mixed with.
            // exclusive pair offsets of edge (a, lane) among the tail-class pairs (po) and the
            // hub-class pairs (ph): each non-decreasing in edge order, an edge of the other class
            // counting 0 pairs (the search takes the last edge at or below a pair's index)
            uint32_t po[UA], ph[UA];
            uint32_t npt = 0, nph = 0;  // tail-class, hub-class pairs
#pragma unroll
            for (int a = 0; a < UA; a++) {
                const uint32_t c = (uint32_t)__popc(amk[a]);
                const bool tl = (an[a] & (g.tflags ? 0x3FFFFFFFu : 0x7FFFFFFFu)) >= D.H;
                uint32_t tt, th = 0;
                po[a] = npt + wave_excl_scan(tl ? c : 0u, &tt);
                ph[a] = nph + wave_excl_scan(tl ? 0u : c, &th);
                npt += tt;
                nph += th;
            }
            const uint32_t rT = (npt + 63u) / 64u;               // tail rounds
            const uint32_t nround = rT + (nph + 63u) / 64u;      // then hub rounds
            // the edge's data for the shuffles: (col | tree bit), (chunk slot | mask << 16)
            uint32_t alm[UA];
#pragma unroll
            for (int a = 0; a < UA; a++) alm[a] = alo[a] | (amk[a] << 16);
            BT_TICK(1);
#if SHD_BATCH_TIME
            if (lane == 0) {
                atomicAdd(&L.bt[6], (unsigned long long)nround);
                atomicAdd(&L.bt[7], (unsigned long long)(npt + nph));
            }
#endif
            uint32_t fm = kNoBucket;
            for (uint32_t r0 = 0; r0 < nround; r0 += RB) {
            uint32_t n[RB], lo[RB], jr[RB], er[RB];
            unsigned long long ab[RB], cur[RB];  // ab = ~0: no pair in this lane
            float kz[RB];                         // kappa0 of the edge's target
            uint32_t tree[RB];
#pragma unroll
            for (int rr = 0; rr < RB; rr++) {
                // round r (uniform): class tail below rT, else hub; q = the pair in its class
                const uint32_t r = r0 + (uint32_t)rr;
                const bool hubr = r >= rT;
                const uint32_t q = (hubr ? r - rT : r) * 64u + lane;
                const uint32_t lim = r >= nround ? 0u : hubr ? nph : npt;
                // last edge E (of UA * 64) whose offset in the round's class is <= q (uniform
                // shuffles, per-lane index)
                uint32_t pc[UA];
#pragma unroll
                for (int a = 0; a < UA; a++) pc[a] = hubr ? ph[a] : po[a];
                uint32_t e = 0;
#pragma unroll
                for (uint32_t st = (uint32_t)UA * 32u; st >= 1u; st >>= 1) {
                    const uint32_t c = e + st;
                    uint32_t oc = 0;
#pragma unroll
                    for (int a = 0; a < UA; a++) {
                        const uint32_t x = __shfl(pc[a], (int)(c & 63u), 64);
                        if ((c >> 6) == (uint32_t)a) oc = x;
                    }
                    if (oc <= q) e = c;
                }
                const int el = (int)(e & 63u);
                uint32_t xn = 0, xlm = 0, xwl = 0, xwh = 0, xpb = 0, xo = 0;
#pragma unroll
                for (int a = 0; a < UA; a++) {
                    const uint32_t t0 = __shfl(an[a], el, 64), t1 = __shfl(alm[a], el, 64);
                    const uint32_t t2 = __shfl(awl[a], el, 64), t3 = __shfl(awh[a], el, 64);
                    const uint32_t t4 = kKapInRec ? __shfl(apb[a], el, 64) : 0u;
                    const uint32_t t5 = __shfl(pc[a], el, 64);
                    if ((e >> 6) == (uint32_t)a) {
                        xn = t0; xlm = t1; xwl = t2; xwh = t3; xpb = t4; xo = t5;
                    }
                }
                bool on = q < lim;
                // source: the (q - offset)-th set bit of the edge's mask
                uint32_t mk = xlm >> 16, k = q - xo, jj = 0;
#pragma unroll
                for (uint32_t wdt = (uint32_t)K / 2u; wdt >= 1u; wdt >>= 1) {
                    const uint32_t c = (uint32_t)__popc(mk & ((1u << wdt) - 1u));
                    if (k >= c) { k -= c; jj += wdt; mk >>= wdt; }
                }
                jr[rr] = jj;
                n[rr] = xn & (g.tflags ? 0x3FFFFFFFu : 0x7FFFFFFFu);
                tree[rr] = xn >> 31;  // the h0-tree edge into n
                lo[rr] = xlm & 0xFFFFu;
                const double w = __hiloint2double((int)xwh, (int)xwl);
                const double abd = __dadd_rn(L.val[lo[rr] * K + jj], w);
                if (kKapInRec) kz[rr] = rec_kap0(xpb);
                er[rr] = on ? e : 0x10000u + lane;  // segment key (no segment across empty lanes)
                ab[rr] = on ? d2bits(abd) : ~0ull;
                // pre-check: the edge's pairs read its target's line in one request
                const bool t = on && n[rr] >= D.H;
                rl_count(L, RL_RELAX_PRE, t, D.dist + (t ? (size_t)n[rr] : (size_t)0) * K + jj);
                const unsigned long long x = D.dist[(t ? (size_t)n[rr] : (size_t)0) * K + jj];
#if SHD_BATCH_TIME
                {
                    const unsigned long long tb = __ballot(t), hb = __ballot(on && !t);
                    if (lane == 0) {
                        if (tb) atomicAdd(&L.sw[0], 1ull);
                        atomicAdd(&L.sw[1], (unsigned long long)__popcll(tb));
                        atomicAdd(&L.sw[2], (unsigned long long)__popcll(hb));
                    }
                }
#endif
                if (!kKapInRec) kz[rr] = g.kap0[t ? n[rr] : 0u];
                cur[rr] = t ? x : 0ull;
            }
            // Tail pairs: the queue bookkeeping (near mask, pending and touched bits) is issued in
            // the same round trip as the returning atomicMin, decided on the pre-check value:
            // a pair that improves now (ab < old <= cur) also had ab < cur, so the speculative
            // bits cover every real one; a spurious bit (a concurrent relaxation lowered the
            // line in between) only re-expands a vertex at its current value, resets an extra
            // line or leaves an extra pending bit -- label-correcting, the fixpoint and every
            // tie / parent hint (decided on the atomic's return) are unchanged.  All RB rounds'
            // atomics are in flight together.
            unsigned long long old[RB];
            uint32_t pm[RB];  // the mask word's previous bits (first: push), or ~0: no mask op
            bool hfv[RB];     // a hub's first deferral
#pragma unroll
            for (int rr = 0; rr < RB; rr++) {
                const bool on = ab[rr] != ~0ull;
                const uint32_t jj = jr[rr];
                const bool hub = n[rr] < D.H;
                bool nr = false, nf = false, ft = false;
                old[rr] = ~0ull;
                if (on && hub) {
                    const size_t wi = (size_t)n[rr] * K + jj;
                    const unsigned long long o = atomicMin(&D.hd[wi], ab[rr]);
                    const bool im = ab[rr] < o;
                    if (im) atomicAnd(&D.xb[wi >> 5], ~(1u << (wi & 31)));
                    if (n[rr] < D.P) {  // parent hint (see the parent pass)
                        wl_count(L, WL_HUB, im, D.hpar + wi);
                        if (im) D.hpar[wi] = L.vx[lo[rr]];
                        else if (ab[rr] == o) atomicOr(&D.tb[wi >> 5], 1u << (wi & 31));
                    }
                    if (im) {
                        const uint32_t b = bkt(bits2d(ab[rr]), L.sh[jj], B.inv_delta);
                        if (b <= B.cb) nr = true;
                        else fm = b < fm ? b : fm;
                    }
                } else if (on && ab[rr] <= cur[rr]) {
                    // the edge's pairs: one coalesced atomic request per line (returning: one
                    // relaxation per value is its improver, every other one producing the same
                    // value a tie -- see the consuming loop)
                    wl_count(L, WL_RELAX_MIN, true, &D.dist[(size_t)n[rr] * K + jj]);
                    old[rr] = atomicMin(&D.dist[(size_t)n[rr] * K + jj], ab[rr]);
                    if (ab[rr] < cur[rr]) {
                        const uint32_t b = bkt(bits2d(ab[rr]), L.sh[jj], B.inv_delta);
                        const bool inf = cur[rr] == kInfBits;
                        ft = inf;
                        if (b <= B.cb) nr = kappa_useful(kz[rr], L.dh0[jj], bits2d(ab[rr]), g.piMax);
                        else nf = inf;
                    }
                }
                uint32_t gm = nr ? 1u << jj : 0u, gf = (nf ? 1u : 0u) | (ft ? 2u : 0u);
#pragma unroll
                for (int o = 1; o < K; o <<= 1) {
                    const uint32_t ym = __shfl_down(gm, o, 64), yf = __shfl_down(gf, o, 64);
                    const uint32_t ye = __shfl_down(er[rr], o, 64);
                    if (lane + (uint32_t)o < 64u && ye == er[rr]) { gm |= ym; gf |= yf; }
                }
                const uint32_t pe = __shfl_up(er[rr], 1, 64);
                const bool head = on && (lane == 0 || pe != er[rr]);
                // first reach: touched (bit 1), and pending when past cb (bit 0): one atomic
                wl_count(L, WL_RELAX_TOUCH, head && gf, &D.pt[n[rr] >> 4]);
                wl_count(L, WL_RELAX_MASK, head && gm && !hub, mnxt + n[rr]);
                if (head && gf) (void)atomicOr(&D.pt[n[rr] >> 4], gf << (2u * (n[rr] & 15u)));
                pm[rr] = ~0u;
                hfv[rr] = false;
                if (head && gm) {
                    if (hub) hfv[rr] = MO::set(hdef, n[rr], gm) == 0u;
                    else pm[rr] = MO::set(mnxt, n[rr], gm);
                }
            }
#pragma unroll
            for (int rr = 0; rr < RB; rr++) {
                const uint32_t jj = jr[rr];
                if (old[rr] != ~0ull) {
                    const size_t wi = (size_t)n[rr] * K + jj;
                    const bool im = ab[rr] < old[rr];
                    // tie: the pair record's tag word := this batch's tag | kTagTie (a plain,
                    // idempotent store; no bitmap to clear for the next batch)
                    wl_count(L, WL_RELAX_TIE, ab[rr] == old[rr], D.tpar + 4 * wi);
                    if (ab[rr] == old[rr]) D.tpar[4 * wi + 1] = B.tie_tag;
                    // the improver: the parent pass' second guess (verified there; the h0-tree
                    // edge needs no record: it is the pass' first guess)
                    wl_count(L, WL_RELAX_HINT, im && !tree[rr], D.tpar + 4 * wi);
                    if (im && !tree[rr]) D.tpar[4 * wi] = L.vx[lo[rr]];
                    if (im) {
                        const uint32_t b = bkt(bits2d(ab[rr]), L.sh[jj], B.inv_delta);
                        if (b > B.cb) fm = b < fm ? b : fm;
                    }
                }
                wpush<K>(L, pm[rr] == 0u, n[rr], qout, &L.qtail, qcap, &L.fover, 1u);
                wpush<K>(L, hfv[rr], n[rr], hq, &L.htail, D.H, &L.fover, 1u);
            }
            }
            if (__ballot(fm != kNoBucket)) {
                fm = wave_min_u32(fm);
                if (lane == 0) atomicMin(&L.fminb, fm);
            }
            BT_TICK(2);
        }
        if (WAVE) {
            // the next sub-chunk overwrites this wave's slice: its lanes' LDS reads are done
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        // this wave's atomics and queue stores complete before any wave reads them after the
        // barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    if (WAVE) {
        // the iteration's atomics and queue stores complete before the next iteration
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

// Load-balanced expansion of a list of (vertex, source) pairs q = v * K + j (parent pass):
// VF(q, val) gives the pair's value, EF(q, val, adjacency slot) handles one edge of v's row.
template <int K, bool DIR, class VF, class EF>
__device__ __forceinline__ void expand_pairs(const uint32_t* Q, uint32_t nq, const DevCSR& g,
                                             LdsB<K>& L, VF&& vf, EF&& ef) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t base = 0; base < nq; base += kBChunk) {
        const uint32_t cnt = min((uint32_t)kBChunk, nq - base);
        uint32_t deg = 0;
        if (tid < cnt) {
            const uint32_t q = Q[base + tid];
            double val = 0.0;
            vf(q, val);
            const uint32_t* rp = DIR ? g.rowptr_in : g.rowptr;  // rows of candidate parents
            const uint32_t r0 = rp[q / K], r1 = rp[q / K + 1];
            deg = r1 - r0;
            L.rs[tid] = r0;
            L.vx[tid] = q;
            L.val[tid] = val;
        }
        uint32_t total;
        const uint32_t off = block_excl_scan<kSsspBlock>(deg, L.wave, &total);
        if (tid < cnt) L.off[tid] = off;
        if (tid == 0) L.off[cnt] = total;
        __syncthreads();
        for (uint32_t e = tid; e < total; e += kSsspBlock) {
            const int lo = chunk_slot<K>(L, cnt, e);
            ef(L.vx[lo], L.val[lo], L.rs[lo] + (e - L.off[lo]));
        }
        __syncthreads();
    }
}

// ---- jobs: a level's parent walks (its start list) and the per-target epilogue are jobs of
// items the workgroup's waves take kJobChunk at a time (round 5 also let idle workgroups join them
// through a help board: measured slower, removed in round 6 -- DESIGN.md 4 item 10)
constexpr uint32_t kJobWalkSync = 1;  // first-level walks (groups of K lanes start together)
constexpr uint32_t kJobWalk = 2;      // later levels
constexpr uint32_t kJobEpi = 3;       // per-target epilogue
constexpr uint32_t kJobChunk = 256;   // items a wave takes at a time
constexpr uint32_t kJobNone = 0xFFFFFFFFu;
constexpr uint32_t kNoPairS = 0xFFFFFFFFu;

}  // namespace

// DIR: a directed topology (parents from the in-rows, DevCSR::rowptr_in); a separate
// instantiation, so the undirected kernel's code and registers are those of round 5 before it.
template <int K, bool DIR>
__global__ void __launch_bounds__(kSsspBlock, kBatchWgPerCu)
sssp_batch_kernel(DevCSR g, SlotWs ws, const uint32_t* __restrict__ sources,
                  const double* __restrict__ srcsh, int nsrc, int kf,
                  const uint32_t* __restrict__ targets, int A, double delta, uint32_t H,
                  uint32_t P, uint32_t iter_guard,
                  double2* __restrict__ out_lr, uint16_t* __restrict__ out_hops,
                  double* __restrict__ out_rowmin, unsigned long long* __restrict__ stats) {
    using MO = MaskOps<K>;
    using M = typename MO::M;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    LdsB<K>& L = *reinterpret_cast<LdsB<K>*>(smem);
    const BLayout lay = blayout<K>(H, P);
    M* hdef = reinterpret_cast<M*>(smem + lay.hdef);
    const uint32_t hmw = (uint32_t)((lay.tb - lay.hdef) / 4);  // u32 words of the hub masks
    const uint32_t tbw = (uint32_t)(((size_t)P * K + 31) / 32);
    const int slot = blockIdx.x;
    const uint32_t tid = threadIdx.x;
    const int64_t V = ws.V;
    BView<K> D;
    D.tb = reinterpret_cast<uint32_t*>(smem + lay.tb);
    D.xb = reinterpret_cast<uint32_t*>(smem + lay.xb);
    const uint32_t xbw = (uint32_t)(((size_t)H * K + 31) / 32);
    D.hd = reinterpret_cast<unsigned long long*>(smem + lay.hd);
    D.dist = ws.dist + (size_t)slot * (size_t)V * K;
    D.hpar = ws.hpar + (size_t)slot * (size_t)P * K;
    D.H = H;
    D.P = P;
    const size_t mbytes = ((size_t)V * sizeof(M) + 255) / 256 * 256;
    M* mA = reinterpret_cast<M*>(ws.mask + (size_t)slot * 2 * mbytes);
    M* mB = reinterpret_cast<M*>(ws.mask + (size_t)slot * 2 * mbytes + mbytes);
    uint32_t* qa = reinterpret_cast<uint32_t*>(ws.qa + (size_t)slot * ws.q_stride);
    uint32_t* qb = reinterpret_cast<uint32_t*>(ws.qb + (size_t)slot * ws.q_stride);
    // parent-pass state per (vertex, source) pair q = v * K + j: the pair record {parent vertex
    // (| amb << 31 | bad << 30), claim tag (the batch that resolved it), f64 loss of the parent
    // edge} -- one 16-B line access per hop of a walk or of the epilogue -- and the row-scan
    // (the row scans' records: ws.rscan, rs_chunk K per slot -- round 5 kept [V][K] arrays of
    // them per slot, 32 GB at C4)
    uint4* prec = ws.prec + (size_t)slot * V * K;
    uint32_t* precw = reinterpret_cast<uint32_t*>(prec);
    D.tpar = precw;
    double* pbuf = ws.pathbuf + (size_t)slot * kPathBufPerSlot;
    uint32_t* ctr = ws.counters + (size_t)slot * 4;
    const uint32_t cap = (uint32_t)V;
    BBuckets B;
    B.inv_delta = 1.0 / delta;
    // parent-pass pair lists: qa / qb (pcur / pnxt) and the ring memory (fscr), V * K entries each,
    // then the merged vertex list
    uint32_t* fscr = reinterpret_cast<uint32_t*>(ws.ring) + (size_t)slot * ws.ring_entries;
    uint32_t* vscr = fscr + (size_t)V * K;  // parent-pass vertex list (V entries)
    // pending / touched bits, 8-B aligned (the ring keeps 64 words of slack per bitmap): the
    // sweeps and the reset read them as pw pairs of words, 32 vertices per pair
    D.pt = reinterpret_cast<uint32_t*>((reinterpret_cast<uintptr_t>(vscr + (size_t)V) + 7) &
                                       ~(uintptr_t)7);
    const uint32_t pw = (uint32_t)((V + 31) / 32);  // word pairs of the pending / touched bits
    unsigned long long* const pt2 = reinterpret_cast<unsigned long long*>(D.pt);
    constexpr unsigned long long kPendBits = 0x5555555555555555ull;
    const uint32_t pcap = (uint32_t)(V * K);

    uint32_t iter = ctr[0];
    if (tid < 4) L.cnt[tid] = 0;
    if (tid < 5) L.pt[tid] = 0;
    if (tid < 4) L.dg[tid] = 0;
    if (tid < 8) L.bt[tid] = 0;
    if (tid < 4) L.sw[tid] = 0;
    if (tid < 16) L.wl[tid] = 0;
    if (tid < 16) L.rl[tid] = 0;
    if (tid == 0) L.touched = 0;
    if (tid < 5) L.wk[tid] = 0;
    if (tid < 4) L.ev[tid] = 0;
    if (tid < 5) L.tm[tid] = 0;
    // phase boundary (all threads pass it together): thread 0 charges the ticks since the last
    // one to phase i
    auto tick = [&](int i) {
        if (tid == 0) {
            const unsigned long long t = wall_clock64();
            L.tm[i] += t - L.tk;
            L.tk = t;
        }
    };

    if (tid == 0) {
        L.jcur = 0;
        L.fover = 0;
    }
    const uint32_t lane = tid & 63u;
    constexpr uint32_t kNoPair = 0xFFFFFFFFu;
    // Walk hop inputs at vertex v for source j: the h0-tree record {parent, slot, f64 w, f64 loss of
    // that edge} (32 B, one line) of a tail and d_j(v) -- independent loads, one round trip.  Hubs
    // read their distance from their row of the [V][K] block (copied there at the SSSP's end).
    struct Hop {
        uint4 sp;
        double sl;
        unsigned long long d;
    };

    // One job of this slot: walks of a level's start list (kJobWalkSync / kJobWalk) or the
    // per-target epilogue (kJobEpi) of the batch {tag epv, positions r0v.., nkv sources}; every
    // wave claims kJobChunk items at a time until the job is used up (L.jcur, reset by the
    // caller).  L.src holds the batch's sources.
    auto run_job = [&](uint32_t kind, uint32_t n, uint32_t epv, uint32_t r0v, uint32_t nkv,
                       uint32_t list) {
        unsigned long long* const distO = D.dist;
        uint4* const precO = prec;
        uint32_t* const precwO = precw;
        const uint32_t eptv = epv | kTagClaim;
        // the wave's next chunk of the job: its first item (kJobNone: used up) and *cnt items
        auto grab = [&](uint32_t* cnt) -> uint32_t {
            uint32_t b = kJobNone, c = 0;
            if (lane == 0) {
                const uint32_t x = atomicAdd(&L.jcur, kJobChunk);
                if (x < n) {
                    b = x;
                    c = min(kJobChunk, n - x);
                }
            }
            *cnt = __shfl(c, 0, 64);
            return __shfl(b, 0, 64);
        };
        if (kind != kJobEpi) {
            // Walks: chains are followed towards the source while the h0-tree guess certifies
            // parents (no level barriers); a chain stops at the source, at a pair another walk
            // claimed first (tag), or at a pair whose guess fails (-> the slot's S list, claimed:
            // the owner's hint pass resolves it).  One round trip per hop: the tag word of q (claim,
            // tie) goes out with the loads of q's tree parent pu (d_j(pu) certifies the guess, pu's
            // own hop inputs serve the next hop).  Flattened: a lane takes its next start pair as
            // soon as its chain ends.  The first level keeps a target's K lanes together (a group
            // takes its next start pairs when the whole group is idle).
            const uint32_t* P = list ? qb : qa;
            uint32_t* const S = fscr;
            const uint32_t pcapS = (uint32_t)(V * K);
            const bool gs = kind == kJobWalkSync;
            auto put = [&](uint32_t q, uint32_t u, double loss) {
                const unsigned long long lb = d2bits(loss);
                wl_count(L, WL_PREC, true, precO + q);
                precO[q] = make_uint4(u, eptv, (uint32_t)lb, (uint32_t)(lb >> 32));
            };
            auto load_hop = [&](uint32_t v, uint32_t j) -> Hop {
                Hop hh;
                const uint32_t q = v * K + j;
                rl_count(L, RL_WALK, v >= H, reinterpret_cast<const uint4*>(g.spt) + 2 * (size_t)v);
                rl_count(L, RL_WALK, true, distO + (size_t)q);
                if (v >= H) {
                    const uint4* sp = reinterpret_cast<const uint4*>(g.spt) + 2 * (size_t)v;
                    hh.sp = sp[0];
                    const uint2 l = *reinterpret_cast<const uint2*>(sp + 1);
                    hh.sl = __hiloint2double((int)l.y, (int)l.x);
                } else {
                    hh.sp = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
                    hh.sl = 0.0;
                }
                hh.d = ld_l2_u64(&distO[(size_t)q]);
                return hh;
            };
            uint32_t i = 0, iend = 0, q = 0, j = 0;
            uint32_t nw = 0, nw0 = 0;   // walk steps, of which certified by the tree guess
            bool act = false, fresh = false, more = true;
            Hop h;
            h.sp = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
            h.sl = 0.0;
            h.d = 0ull;
            for (;;) {
                if (more && !__any(i < iend)) {
                    uint32_t c;
                    const uint32_t b = grab(&c);
                    if (b == kJobNone) {
                        more = false;
                    } else {
                        i = b + lane;
                        iend = b + c;
                    }
                }
                bool take = !act && i < iend;
                if (gs) {  // the lane's group of K (one target) takes its starts together
                    const unsigned long long am = __ballot(act);
                    take = take && ((am >> (lane & ~(uint32_t)(K - 1))) & ((1ull << K) - 1ull)) == 0ull;
                }
                rl_count(L, RL_WALK, take, P + (take ? i : 0u));
                if (take) {
                    q = P[i];
                    i += 64;
                    j = q % K;
                    act = q != kNoPair;
                    fresh = act;
                }
                if (!more && !__any(act || i < iend)) break;
                bool sp = false;  // q goes to the S list
                if (act && fresh) {
                    h = load_hop(q / K, j);
                    fresh = false;
                } else if (act) {
                    const uint32_t v = q / K;
                    const uint32_t pu = h.sp.x;
                    const bool tree = v >= H && pu < (uint32_t)V;
                    Hop hn = h;
                    if (tree) hn = load_hop(pu, j);
                    // The claim is a plain tag read issued with those loads; the pair's record
                    // (put) or, for a pair left to the hint pass, a tag store marks it as this
                    // batch's.  Two walks that reach an unclaimed pair in the same round trip both
                    // walk on: they write identical records (the parent rule is deterministic), and
                    // a pair listed twice in S is resolved twice the same way.
                    rl_count(L, RL_WALK, true, precwO + 4 * (size_t)q);
                    const uint32_t tw = ld_l2_u32(&precwO[4 * (size_t)q + 1]);
                    if (tag_claimed(tw, epv)) {  // another walk's
                        act = false;
                    } else {
                        nw++;
                        const bool tied = tag_tied(tw, epv);
                        if (tree && !tied &&
                            __dadd_rn(bits2d(hn.d), __hiloint2double((int)h.sp.w, (int)h.sp.z)) ==
                                bits2d(h.d)) {
                            put(q, pu, h.sl);
                            nw0++;
                            if (pu == L.src[j]) {
                                act = false;
                            } else {
                                q = pu * K + j;
                                h = hn;
                            }
                        } else {
                            wl_count(L, WL_PREC, true, precwO + 4 * (size_t)q);
                            precwO[4 * (size_t)q + 1] = eptv | (tied ? kTagTie : 0u);
                            sp = true;
                            act = false;
                        }
                    }
                }
                // this round's S pairs, wave-aggregated
                const unsigned long long m = __ballot(sp);
                if (m) {
                    const uint32_t need = (uint32_t)__popcll(m);
                    uint32_t x = 0;
                    if (lane == 0) x = atomicAdd(&L.qtail, need);
                    const uint32_t base = __shfl(x, 0, 64);
                    if (sp) {
                        const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                        wl_count(L, WL_QUEUE, pos < pcapS, S + pos);
                        if (pos < pcapS) S[pos] = q;
                        else atomicOr(&L.fover, 128u);
                    }
                }
            }
            const unsigned long long s0 = wave_sum_u64(nw), s1 = wave_sum_u64(nw0);
            if (lane == 0) {
                atomicAdd(&L.wk[0], s0);
                atomicAdd(&L.wk[1], s1);
            }
        } else {
            // Per-target latency / reliability / hops (shd-topology.c:561-671), items (target,
            // source) target-major (the group's chains coincide up to the core, so each lockstep
            // hop reads one target's pair records); each lane walks its item's chain backwards into
            // its path buffer (the first nl levels in this workgroup's hub LDS, whose distances are
            // in HBM by now; deeper ones in its HBM buffer) and multiplies in path order.
            double* lpb = reinterpret_cast<double*>(smem + lay.hd);
            const uint32_t nl = H * K / kSsspBlock;  // LDS levels of the path buffer
            auto pb_at = [&](uint32_t x) -> double* {
                return x < nl ? lpb + (size_t)x * kSsspBlock + tid : pbuf + (size_t)x * kSsspBlock + tid;
            };
            unsigned long long* const rminP = L.rmin;
            for (;;) {
                uint32_t c;
                const uint32_t b = grab(&c);
                if (b == kJobNone) break;
                for (uint32_t i = b + lane; i < b + c; i += 64) {
                    const uint32_t jj = i % nkv;  // target-major: a target's sources adjacent
                    const uint32_t k = i / nkv;
                    rl_count(L, RL_EPI, true, targets + k);
                    const uint32_t t = targets[k];
                    const uint32_t src = L.src[jj];
                    double lat, rel;
                    uint32_t hcnt = 0;
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
                            hcnt = 1;
                        }
                    } else {
                        rl_count(L, RL_EPI, true, distO + (size_t)t * K + jj);
                        rl_count(L, RL_EPI, true, g.vloss + t);
                        lat = bits2d(ld_l2_u64(&distO[(size_t)t * K + jj]));
                        bool amb = false, bad = false;
                        uint32_t v = t;
                        while (v != src) {
                            // the pair record, L1-bypassing (written by other waves / workgroups)
                            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                            rl_count(L, RL_EPI, true, reinterpret_cast<const u32x4*>(precO) + (size_t)v * K + jj);
                            const u32x4 rv = __builtin_nontemporal_load(
                                reinterpret_cast<const u32x4*>(precO) + (size_t)v * K + jj);
                            if (rv.y != eptv || (rv.x & 0x40000000u)) {
                                bad = true;
                                break;
                            }
                            amb |= (rv.x >> 31) != 0u;
                            wl_count(L, WL_OTHER, hcnt < kMaxHops && hcnt >= nl, pb_at(hcnt));
                            if (hcnt < kMaxHops) *pb_at(hcnt) = __hiloint2double((int)rv.w, (int)rv.z);
                            hcnt++;
                            v = rv.x & 0x3FFFFFFFu;
                            if (hcnt > (uint32_t)V) { bad = true; break; }
                        }
                        rel = 1.0;
                        rel *= (1.0 - g.vloss[src]);
                        rel *= (1.0 - g.vloss[t]);
                        if (bad) {
                            atomicAdd(&stats[ST_ERRORS], 1ull);
                            lat = -1.0;
                            rel = -1.0;
                        } else if (hcnt <= (uint32_t)kMaxHops) {
                            for (int x = (int)hcnt - 1; x >= 0; --x) rel *= (1.0 - *pb_at((uint32_t)x));
                        } else {
                            atomicAdd(&stats[ST_LONGPATH], 1ull);
                            for (int x = (int)hcnt - 1; x >= 0; --x) {  // edge at depth x from t
                                uint32_t y = t;
                                for (int z = 0; z < x; ++z) y = precO[(size_t)y * K + jj].x & 0x3FFFFFFFu;
                                const uint4 r = precO[(size_t)y * K + jj];
                                rel *= (1.0 - __hiloint2double((int)r.w, (int)r.z));
                            }
                        }
                        if (amb) {
                            atomicAdd(&stats[ST_AMBIGUOUS], 1ull);
                            if (ws.rowflag) ws.rowflag[ws.rowmap ? ws.rowmap[r0v + jj] : r0v + jj] = 1;  // tie replay (topo_replay.hip)
                        }
                        if (lat == 0.0) lat = 1.0;
                    }
                    const size_t ob = (size_t)(ws.rowmap ? (int)ws.rowmap[r0v + jj] : (int)(r0v + jj)) * (size_t)A + k;
                    const uint16_t hh = (uint16_t)(hcnt > 65535u ? 65535u : hcnt);
                    wl_count(L, WL_OUT, true, out_lr + ob);
                    wl_count(L, WL_OUT, true, out_hops + ob);
                    {  // the table (1.8 GB per launch) is not re-read by the kernel: nontemporal
                        typedef double f64x2 __attribute__((ext_vector_type(2)));
                        const f64x2 r2 = {lat, rel};
                        __builtin_nontemporal_store(r2, reinterpret_cast<f64x2*>(out_lr) + ob);
                        __builtin_nontemporal_store(hh, out_hops + ob);
                    }
                    if (lat >= 0.0) atomicMin(&rminP[jj], d2bits(lat));  // row minimum (runahead)
                }
            }
        }
    };

    for (;;) {
        if (tid == 0) L.idx = (uint32_t)atomicAdd(&stats[ST_DEQUEUE], 1ull);
        __syncthreads();
        const uint32_t bidx = L.idx;
        __syncthreads();
        // batch bidx: sources [bidx kf, bidx kf + kf) in lanes 0..nk-1 (kf <= K: the host fills
        // batches below K when that finishes the sources in fewer rounds of the slots), or the
        // host's layout [bstart[bidx], bstart[bidx + 1]) sized by measured costs
        int r0, nk;
        if (ws.bstart) {
            if (bidx >= (uint32_t)ws.nbat) break;
            r0 = (int)ws.bstart[bidx];
            nk = (int)ws.bstart[bidx + 1] - r0;
        } else {
            if ((int64_t)bidx * kf >= nsrc) break;
            r0 = (int)bidx * kf;
            nk = min(kf, nsrc - r0);
        }
        if (tid == 0) L.tk = wall_clock64();
        if (ws.btrace && tid == 0) {
            ws.btrace[kBTraceWords * (size_t)bidx] = L.tk;
            ws.btrace[kBTraceWords * (size_t)bidx + 3] = L.ev[0];
            ws.btrace[kBTraceWords * (size_t)bidx + 4] = L.ev[1];
            ws.btrace[kBTraceWords * (size_t)bidx + 5] = L.ev[2];
            ws.btrace[kBTraceWords * (size_t)bidx + 6] = L.cnt[0];
            ws.btrace[kBTraceWords * (size_t)bidx + 2] = (unsigned long long)slot;
        }

        // ---------------- init: hubs in LDS, the tail's K-wide rows in HBM --------------------
        for (uint32_t i = tid; i < H * K; i += kSsspBlock) D.hd[i] = kInfBits;
        for (uint32_t i = tid; i < hmw; i += kSsspBlock) {
            reinterpret_cast<uint32_t*>(hdef)[i] = 0u;
        }
        for (uint32_t i = tid; i < tbw; i += kSsspBlock) D.tb[i] = 0u;
        for (uint32_t i = tid; i < xbw; i += kSsspBlock) D.xb[i] = 0u;
        // (the pending / touched words are zero: the previous batch's reset cleared every word
        // it touched, and a pending vertex is always touched)
        // the batch's tag: claims of the parent pass, ties of the SSSP (pair records)
        iter++;
        const uint32_t ep = (iter - 1u) % kTagMask + 1u;
        B.tie_tag = ep | kTagTie;
        if (tid < (uint32_t)K) L.sh[tid] = (int)tid < nk ? srcsh[r0 + tid] : 0.0;
        // no landmark bound until h0 is reached (the sweeps test kappa0 against L.dh0)
        if (tid < (uint32_t)K) L.dh0[tid] = INFINITY;
        if (tid == 0) L.invd = B.inv_delta;
        if (tid == 0) {
            L.fminb = kNoBucket;
            L.fover = 0;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // every source starts at its own (shifted) bucket: found by the first sweep
        if ((int)tid < nk) {
            const uint32_t s = sources[r0 + tid];
            if (s < H) D.hd[(size_t)s * K + tid] = 0ull;
            else {
                D.dist[(size_t)s * K + tid] = 0ull;
                atomicOr(&D.pt[s >> 4], 3u << (2u * (s & 15u)));
            }
            atomicMin(&L.fminb, bkt(0.0, L.sh[tid], B.inv_delta));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        tick(0);

        // ---------------- lock-step delta-stepping over the shifted buckets -------------------
        // L.fminb is exact at every bucket change: the sweep sets it to the smallest pending
        // bucket past the one it opens, and every improvement past cb lowers it.
        B.cb = 0;
        M* mcur = mA; M* mnxt = mB;
        uint32_t* qin = qa; uint32_t* qout = qb;
        uint32_t* hfill = qa + V;  // deferred hub list being filled
        uint32_t* hdrain = qb + V; // ... and the one being expanded
        uint32_t nq = 0;
        uint32_t guard = 0;
        bool aborted = false;
        bool just_swept = false;
        if (tid == 0) L.htail = 0;
        __syncthreads();
        for (;;) {
            // near phase of bucket cb: tail iterations until the tail queue is empty, then one
            // iteration over the deferred hubs, until neither has work
            for (;;) {
                const uint32_t nh = L.htail;
                const bool hubs = nq == 0;
                if (hubs && nh == 0) break;
                if (hubs) { uint32_t* t = hfill; hfill = hdrain; hdrain = t; }
                const uint32_t* src = hubs ? hdrain : qin;
                const uint32_t ns = hubs ? min(nh, H) : nq;
                __syncthreads();
                if (tid == 0) {
                    L.qtail = 0;
                    L.qhead = 0;
                    if (hubs) L.htail = 0;
                }
                __syncthreads();
                if (tid == 0) L.ev[2] += ns;
                const unsigned long long e0 = L.cnt[2], a0 = L.cnt[0];
                const bool first_it = guard == 0 || just_swept;
                if (!hubs)
                    relax_batch_t<K, kBatchU, true>(src, ns, g, L, D, mcur, hdef, mnxt, qout,
                                                    cap, hfill, B);
                else
                    relax_batch_t<K, kBatchU>(src, ns, g, L, D, mcur, hdef, mnxt, qout, cap,
                                              hfill, B);
                nq = min(L.qtail, cap);
                if (tid == 0 && first_it) {
                    L.dg[2] += L.cnt[2] - e0;
                    L.dg[3] += L.cnt[0] - a0;
                }
                just_swept = false;
                { uint32_t* t = qin; qin = qout; qout = t; }
                { M* t = mcur; mcur = mnxt; mnxt = t; }
                if (tid == 0) L.ev[0]++;
                if (++guard > iter_guard) {
                    aborted = true;
                    nq = 0;
                    break;
                }
                __syncthreads();
            }
            if (aborted) break;
            const uint32_t nb = L.fminb;
            if (nb == kNoBucket) break;  // nothing pending: the batch is settled
            const unsigned long long ts0 = wall_clock64();
            // Sweep: classify every (vertex, source) word by its bucket (K / 2 lanes per vertex,
            // 16 B each); the pairs of bucket nb form the near queue with their masks in mcur
            // (hubs: the deferred list, masks in hdef; all zero here), the smallest bucket past
            // nb becomes L.fminb.
            __syncthreads();
            if (tid == 0) {
                L.qtail = 0;
                L.fminb = kNoBucket;
            }
            __syncthreads();
            {
                static_assert(K >= 2 && 64 % (K / 2) == 0, "lanes per vertex");
                constexpr uint32_t LPV = K / 2;
                const size_t hpair = (size_t)H * K / 2;
                constexpr int SU = 8;  // 16-B loads in flight per lane (8 > 4 by 0.3 %, 2: +0.8 %)
                // hubs: every (hub, source) word of LDS
                for (size_t ib = 0; ib < hpair; ib += (size_t)kSsspBlock * SU) {
                    unsigned long long d[SU][2];
#pragma unroll
                    for (int u = 0; u < SU; u++) {
                        const size_t i = ib + (size_t)u * kSsspBlock + tid;
                        d[u][0] = d[u][1] = kInfBits;
                        if (i < hpair) {
                            d[u][0] = D.hd[2 * i];
                            d[u][1] = D.hd[2 * i + 1];
                        }
                    }
                    uint32_t km = kNoBucket;
#pragma unroll
                    for (int u = 0; u < SU; u++) {
                        const size_t i = ib + (size_t)u * kSsspBlock + tid;
                        const uint32_t jl = (uint32_t)((2 * i) % K);
                        uint32_t m = 0;
#pragma unroll
                        for (int h = 0; h < 2; h++) {
                            if (d[u][h] == kInfBits) continue;
                            // a hub pair expanded (speculatively) at its current value is done
                            if ((D.xb[(2 * i + h) >> 5] >> ((2 * i + h) & 31)) & 1u) continue;
                            const uint32_t b = bkt(bits2d(d[u][h]), L.sh[jl + h], B.inv_delta);
                            if (b == nb) m |= 1u << (jl + h);
                            else if (b > nb && b < km) km = b;
                        }
#pragma unroll
                        for (uint32_t o = 1; o < LPV; o <<= 1) m |= __shfl_xor(m, (int)o, 64);
                        const uint32_t v = (uint32_t)(2 * i / K);
                        const bool lead = (tid % LPV) == 0 && m != 0u && i < hpair;
                        if (lead) hdef[v] = (M)m;
                        wpush<K>(L, lead, v, hfill, &L.htail, H, &L.fover, 32u);
                    }
                    km = wave_min_u32(km);
                    if ((tid & 63) == 0 && km != kNoBucket) atomicMin(&L.fminb, km);
                }
                // tail: only the vertices whose pending bit is set (~9 % of them per sweep on
                // C4, instead of streaming all [V][K] rows).  A round takes one bitmap word per
                // thread, compacts the set bits' vertices into LDS (the chunk buffers are idle
                // here), classifies their lines (LPV lanes x 16 B per vertex) and rewrites the
                // words with the vertices that still hold a pair past nb.
                // Wave-parallel tail sweep: every wave owns blocks of SG x 64 word pairs (SG per
                // lane, 32 vertices each), compacts their pending bits into its own LDS slice,
                // classifies those lines and rewrites its own words -- no block barrier until the
                // sweep ends.  ~1.7 % of the vertices are pending per sweep, so a block of 64
                // word pairs yields ~35 vertices; SG blocks share one round trip of line loads.
                {
                    constexpr uint32_t SG = 2;  // word pairs per lane and block (2: -2.9 %; 4 spills)
                    constexpr uint32_t NW = kSsspBlock / 64;
                    constexpr uint32_t VPW = 64 / LPV;  // vertices per wave instruction
                    constexpr uint32_t kKeep = 0x80000000u;  // slice entry: the vertex stays pending
                    // the chunk buffers (off .. val, contiguous and idle here): each wave's
                    // compaction slice
                    constexpr uint32_t kSweepU32 =
                        (uint32_t)((offsetof(LdsB<K>, val) + sizeof(L.val) - offsetof(LdsB<K>, off)) / 4);
                    constexpr uint32_t kClW = kSweepU32 / NW;
                    static_assert(kClW >= 64, "sweep compaction slice");
                    const uint32_t wv = tid >> 6, lane = tid & 63u;
                    uint32_t* clw = L.off + wv * kClW;
                    const uint32_t w0 = H / 32;
                    unsigned long long nword[SG];
#pragma unroll
                    for (uint32_t gi = 0; gi < SG; gi++) {
                        const uint32_t wi = w0 + wv * 64u * SG + gi * 64u + lane;
                        nword[gi] = wi < pw ? ld_l2_u64(&pt2[wi]) : 0ull;
                    }
                    for (uint32_t bb = w0 + wv * 64u * SG; bb < pw; bb += NW * 64u * SG) {
                        unsigned long long word[SG], surv[SG];
                        uint32_t cnt = 0;
#pragma unroll
                        for (uint32_t gi = 0; gi < SG; gi++) {
                            word[gi] = nword[gi];
                            surv[gi] = 0ull;
                            cnt += (uint32_t)__popcll(word[gi] & kPendBits);
                            const uint32_t wn = bb + NW * 64u * SG + gi * 64u + lane;
                            rl_count(L, RL_SWEEP, wn < pw, pt2 + (wn < pw ? wn : 0u));
                            nword[gi] = wn < pw ? ld_l2_u64(&pt2[wn]) : 0ull;
                        }
                        uint32_t tot;
                        const uint32_t off = wave_excl_scan(cnt, &tot);
                        for (uint32_t p0 = 0; p0 < tot; p0 += kClW) {
                            {
                                uint32_t o = off;
#pragma unroll
                                for (uint32_t gi = 0; gi < SG; gi++) {
                                    unsigned long long w = word[gi] & kPendBits;
                                    const uint32_t wi = bb + gi * 64u + lane;
                                    while (w) {
                                        const uint32_t b = (uint32_t)__ffsll((long long)w) - 1u;
                                        w &= w - 1ull;
                                        if (o >= p0 && o < p0 + kClW) clw[o - p0] = wi * 32u + b / 2u;
                                        o++;
                                    }
                                }
                            }
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            __builtin_amdgcn_wave_barrier();
                            const uint32_t n = min(kClW, tot - p0);
                            for (uint32_t vb = 0; vb < n; vb += VPW * SU) {
                                unsigned long long d[SU][2];
                                uint32_t vv[SU];
                                float k0[SU];
#pragma unroll
                                for (int u = 0; u < SU; u++) {
                                    const uint32_t e = vb + (uint32_t)u * VPW + lane / LPV;
                                    vv[u] = e < n ? clw[e] : 0xFFFFFFFFu;
                                    rl_count(L, RL_SWEEP, e < n, reinterpret_cast<const char*>(D.dist) + ((size_t)(e < n ? vv[u] : 0u) * LPV + lane % LPV) * 16);
                                    rl_count(L, RL_SWEEP, e < n, g.kap0 + (e < n ? vv[u] : 0u));
                                    k0[u] = g.kap0[e < n ? vv[u] : 0u];
                                    d[u][0] = d[u][1] = kInfBits;
                                    if (e < n) {
                                        typedef unsigned long long u64x2
                                            __attribute__((ext_vector_type(2)));
                                        const u64x2 x = __builtin_nontemporal_load(
                                            reinterpret_cast<const u64x2*>(D.dist) +
                                            (size_t)vv[u] * LPV + lane % LPV);
                                        d[u][0] = x.x;
                                        d[u][1] = x.y;
                                    }
                                }
                                uint32_t km = kNoBucket;
#pragma unroll
                                for (int u = 0; u < SU; u++) {
                                    const uint32_t jl = 2 * (lane % LPV);
                                    uint32_t m = 0, keep = 0;
#pragma unroll
                                    for (int h = 0; h < 2; h++) {
                                        if (d[u][h] == kInfBits) continue;
                                        const uint32_t b = bkt(bits2d(d[u][h]), L.sh[jl + h],
                                                               B.inv_delta);
                                        if (b == nb) {
                                            if (kappa_useful(k0[u], L.dh0[jl + h],
                                                             bits2d(d[u][h]), g.piMax))
                                                m |= 1u << (jl + h);
                                        } else if (b > nb) {
                                            keep = 1u;
                                            if (b < km) km = b;
                                        }
                                    }
#pragma unroll
                                    for (uint32_t o = 1; o < LPV; o <<= 1) {
                                        m |= __shfl_xor(m, (int)o, 64);
                                        keep |= __shfl_xor(keep, (int)o, 64);
                                    }
                                    const uint32_t v = vv[u];
                                    const uint32_t e = vb + (uint32_t)u * VPW + lane / LPV;
                                    const bool ok = (lane % LPV) == 0 && v != 0xFFFFFFFFu;
                                    const bool lead = ok && m != 0u;
                                    wl_count(L, WL_MASK_ST, lead, mcur + (lead ? v : 0u));
                                    if (lead) mcur[v] = (M)m;
                                    if (ok && keep) clw[e] = v | kKeep;
                                    wpush<K>(L, lead, v, qin, &L.qtail, cap, &L.fover, 32u);
                                }
                                km = wave_min_u32(km);
                                if (lane == 0 && km != kNoBucket) atomicMin(&L.fminb, km);
                            }
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            __builtin_amdgcn_wave_barrier();
                            // this pass's survivors back into the lanes' words (same bit order)
                            {
                                uint32_t o = off;
#pragma unroll
                                for (uint32_t gi = 0; gi < SG; gi++) {
                                    unsigned long long w = word[gi] & kPendBits;
                                    while (w) {
                                        const uint32_t b = (uint32_t)__ffsll((long long)w) - 1u;
                                        w &= w - 1ull;
                                        if (o >= p0 && o < p0 + kClW && (clw[o - p0] & kKeep))
                                            surv[gi] |= 1ull << b;
                                        o++;
                                    }
                                }
                            }
                            // the slice is refilled by the next pass
                            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                            __builtin_amdgcn_wave_barrier();
                        }
                        // the touched bits stay; surv holds a subset of the pending bits: an
                        // unchanged pair needs no store
#pragma unroll
                        for (uint32_t gi = 0; gi < SG; gi++) {
                            const uint32_t wi = bb + gi * 64u + lane;
                            const unsigned long long nw = (word[gi] & ~kPendBits) | surv[gi];
                            wl_count(L, WL_PEND_ST, wi < pw && nw != word[gi], pt2 + wi);
                            if (wi < pw && nw != word[gi]) pt2[wi] = nw;
                        }
                    }
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            nq = min(L.qtail, cap);
            if (tid == 0) L.cnt[1] += nq;
            B.cb = nb;
            just_swept = true;
            if (tid == 0) {
                L.ev[1]++;
                L.tm[4] += wall_clock64() - ts0;
            }
            __syncthreads();
        }
        if (aborted) {
            // iteration guard: leave the masks clean for the next batch and report
            for (size_t i = tid; i < 2 * mbytes / 4; i += kSsspBlock)
                reinterpret_cast<uint32_t*>(mA)[i] = 0u;
            if (tid == 0) atomicOr(&stats[ST_OVERFLOW], 2ull);
            __syncthreads();
        }
        if (tid == 0 && L.fover) {
            atomicAdd(&stats[ST_FARSCAN], 1ull);
            atomicOr(&stats[ST_OVERSITE], (unsigned long long)L.fover);
        }
        tick(1);
        if (ws.btrace && tid == 0) ws.btrace[kBTraceWords * (size_t)bidx + 8] = L.tk;

        // ---------------- parents for the target chains of every source of the batch ---------
        // One level-synchronous pass over (vertex, source) pairs p = v * K + j (SURVEY.md A.3:
        // parent(v) = argmin d_j[u] over the candidates fl(d_j[u] + w) == d_j[v]).  A level's walks
        // certify most parents without scanning (h0-tree guess); the rest get the hint pass and a
        // merged row scan; their parents start the next level.  Each level's walks and the
        // epilogue are jobs (run_job) the workgroup's waves take in chunks.
        if ((int)tid < nk) L.src[tid] = sources[r0 + tid];
        const uint32_t ept = ep | kTagClaim;  // tag word of a resolved / claimed pair record
        // A job starts once every wave's earlier stores are drained (the hub rows, the start
        // list, the pair records), and ends when every wave's stores are.
        auto job_start = [&](uint32_t kind) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                L.jcur = 0;
                L.qtail = 0;
                if (kind == kJobEpi)
                    for (int jj = 0; jj < K; jj++) L.rmin[jj] = kInfBits;
            }
            __syncthreads();
        };
        auto job_end = [&]() {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        };
        // the hub distances move to their (otherwise unused) rows of the [V][K] block: the walks
        // and the epilogue of every workgroup taking part in this batch's jobs read them there
        for (uint32_t i = tid; i < H * K; i += kSsspBlock) {
            wl_count(L, WL_HUB, true, D.dist + i);
            D.dist[i] = D.hd[i];
        }
        if (tid == 0) L.qtail = 0;
        __syncthreads();
        uint32_t* pcur = qa;
        uint32_t* pnxt = qb;
        uint32_t plist = 0;  // pcur is qa (0) or qb (1)
        // Target-major start list, K entries per target (kNoPair for the sources past nk and a
        // target that is the source): a target's chains for the K sources share their tail part
        // (the h0-tree guess is source-independent), so the K lanes of an aligned group walk the
        // same vertices in the same round trip and one line serves the group's tree records,
        // distances and pair records.  The first level's walks keep the groups together (a lane
        // takes its next start pair when its whole group is idle).
        for (uint32_t i = tid; i < (uint32_t)A * K; i += kSsspBlock) {
            const uint32_t j = i % K;
            const uint32_t t = targets[i / K];
            const bool p = j < (uint32_t)nk && t != L.src[j];
            wl_count(L, WL_QUEUE, true, pcur + i);
            pcur[i] = p ? t * K + j : kNoPair;
        }
        uint32_t nF = (uint32_t)A * K;
        uint32_t wkind = kJobWalkSync;
        // A pair's record: its parent, the batch's tag, the loss of the parent edge (one store)
        auto put = [&](uint32_t q, uint32_t u, double loss) {
            const unsigned long long lb = d2bits(loss);
            wl_count(L, WL_PREC, true, prec + q);
            prec[q] = make_uint4(u, ept, (uint32_t)lb, (uint32_t)(lb >> 32));
        };
        // A guess certified without scanning a row, past the h0-tree guess of a tail (tried by
        // the walk itself): a tail's recorded improver u (no tie bit; the edge is found in v's own
        // row -- a tail: short -- the same undirected edge, same latency and loss as u's slot) or
        // the first P hubs' recorded improver (LDS hint, no tie bit; the edge in u's row).  The
        // hint pass runs two pairs per thread with their dependent loads interleaved (record ->
        // row bounds and d_j(u) -> binary search -> edge record and loss): half the serial round
        // trips of one pair at a time.  A certified pair's record is written (put).
        constexpr int kHP = 2;  // pairs per thread in flight
        auto hint_pass = [&](const uint32_t* S, uint32_t nS, uint32_t ib, bool* scan, uint32_t* qo) {
            uint32_t q[kHP], uu[kHP], key[kHP], lo[kHP], hi[kHP], end[kHP];
            unsigned long long dv[kHP], du[kHP];
            bool has[kHP], live[kHP];
            uint2 rw[kHP];
            uint32_t hp[kHP], tbit[kHP];
#pragma unroll
            for (int h = 0; h < kHP; h++) {
                const uint32_t i = ib + (uint32_t)h * kSsspBlock + tid;
                q[h] = i < nS ? S[i] : kNoPairS;
                has[h] = q[h] != kNoPairS;
                qo[h] = q[h];
                if (!has[h]) q[h] = 0u;
                const uint32_t v = q[h] / K, j = q[h] % K;
                dv[h] = has[h] ? D.get(v, j) : 0ull;
                rw[h] = make_uint2(0u, 0u);
                hp[h] = 0xFFFFFFFFu;
                tbit[h] = 1u;
                if (has[h] && v >= H) {
                    // the record {improver, tag word} (the walk's tag store kept the tie flag)
                    rw[h] = __hip_atomic_load(reinterpret_cast<const uint2*>(precw + 4 * (size_t)q[h]),
                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                } else if (has[h] && v < P) {
                    tbit[h] = (D.tb[q[h] >> 5] >> (q[h] & 31)) & 1u;
                    hp[h] = D.hpar[q[h]];
                }
            }
#pragma unroll
            for (int h = 0; h < kHP; h++) {
                const uint32_t v = q[h] / K, j = q[h] % K;
                live[h] = false;
                uu[h] = 0xFFFFFFFFu;
                key[h] = 0u;
                uint32_t row = 0;
                if (has[h] && g.rows_sorted) {
                    if (v >= H) {
                        const uint32_t u = rw[h].x & 0x3FFFFFFFu;
                        if (!tag_tied(rw[h].y, ep) && u < (uint32_t)V && u != v) {
                            live[h] = true;
                            uu[h] = u;
                            key[h] = u;
                            row = v;
                        }
                    } else if (v < P && !tbit[h] && hp[h] < (uint32_t)V) {
                        // the edge hint -> hub: found in the hint's row (undirected: usually
                        // far shorter than the hub's), in the hub's in-row when directed
                        live[h] = true;
                        uu[h] = hp[h];
                        key[h] = DIR ? hp[h] : v;
                        row = DIR ? v : hp[h];
                    }
                }
                const uint32_t* rp = DIR ? g.rowptr_in : g.rowptr;
                lo[h] = live[h] ? rp[row] : 0u;
                hi[h] = live[h] ? rp[row + 1] : 0u;
                du[h] = live[h] ? D.get(uu[h], j) : 0ull;
                end[h] = hi[h];
            }
            // binary searches of the rows (sorted by neighbour), side by side
            for (;;) {
                bool any = false;
                uint32_t mid[kHP], c[kHP];
#pragma unroll
                for (int h = 0; h < kHP; h++) {
                    const bool go = live[h] && lo[h] < hi[h];
                    mid[h] = (lo[h] + hi[h]) >> 1;
                    c[h] = go ? adj_col(g, mid[h]) : 0u;
                    any = any || go;
                }
                if (!any) break;
#pragma unroll
                for (int h = 0; h < kHP; h++) {
                    if (!(live[h] && lo[h] < hi[h])) continue;
                    if (c[h] < key[h]) lo[h] = mid[h] + 1u; else hi[h] = mid[h];
                }
            }
#pragma unroll
            for (int h = 0; h < kHP; h++) {
                scan[h] = has[h];
                if (!live[h] || lo[h] >= end[h]) continue;
                const AdjRec ar = adj_rec(g, lo[h]);
                const double ls = g.aloss[lo[h]];
                if (ar.a != key[h]) continue;
                if (__dadd_rn(bits2d(du[h]), rec_wt(ar)) != bits2d(dv[h])) continue;
                put(q[h], uu[h], ls);
                scan[h] = false;
            }
        };
        while (nF > 0) {
            if (tid == 0) L.ev[3] += nF;
            unsigned long long tp0 = wall_clock64();
            job_start(wkind);
            run_job(wkind, nF, ep, (uint32_t)r0, (uint32_t)nk, plist);
            job_end();
            // the S list (pairs whose guess failed)
            const uint32_t nS = min(L.qtail, pcap);
            __syncthreads();
            if (tid == 0) L.pt[1] += wall_clock64() - tp0;  // walks
            if (nS == 0) break;
            tp0 = wall_clock64();
            // hint pass over S (pt[2] with the row scans): the recorded improvers (a tail's, the
            // first P hubs'), in lockstep; the pairs left need a row scan: R, compacted into pcur
            // (consumed by the walks)
            if (tid == 0) L.qtail = 0;
            __syncthreads();
            for (uint32_t ib = 0; ib < nS; ib += (uint32_t)kHP * kSsspBlock) {
                bool scan[kHP];
                uint32_t qs[kHP];
                hint_pass(fscr, nS, ib, scan, qs);
#pragma unroll
                for (int h = 0; h < kHP; h++) {
                    const uint32_t q = qs[h];
                    const bool in = ib + (uint32_t)h * kSsspBlock + tid < nS && q != kNoPairS;
                    // counters (walk kinds): tail hint, hub hint, row scan -- one LDS atomic per wave
                    const unsigned long long bt = __ballot(in && !scan[h] && q / K >= H);
                    const unsigned long long bh = __ballot(in && !scan[h] && q / K < H);
                    const unsigned long long bs = __ballot(in && scan[h]);
                    if ((tid & 63u) == 0u) {
                        if (bt) atomicAdd(&L.wk[2], (unsigned long long)__popcll(bt));
                        if (bh) atomicAdd(&L.wk[3], (unsigned long long)__popcll(bh));
                        if (bs) atomicAdd(&L.wk[4], (unsigned long long)__popcll(bs));
                    }
                    wpush<K>(L, in && scan[h], q, pcur, &L.qtail, pcap, &L.fover, 128u);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const uint32_t nR = min(L.qtail, pcap);
            __syncthreads();
            // R in chunks of ws.rs_chunk pairs (C4: ~2.6 k per level of a batch, one chunk)
            if (tid == 0) L.rsb = 0;
            __syncthreads();
            for (;;) {
                const uint32_t rb = L.rsb;
                if (rb >= nR) break;
                const uint32_t nc = min(ws.rs_chunk, nR - rb);
                const uint32_t* rl = pcur + rb;
                uint4* const rs = ws.rscan + (size_t)slot * ws.rs_chunk * K;
                // merge the pairs by vertex (masks in mA / hdef, zero after the SSSP): a vertex's
                // row is scanned once for every source whose chain needs it
                if (tid == 0) L.qtail = 0;
                __syncthreads();
                for (uint32_t ib = 0; ib < nc; ib += kSsspBlock) {
                    const uint32_t i = ib + tid;
                    bool first = false;
                    uint32_t v = 0;
                    if (i < nc) {
                        const uint32_t q = rl[i];
                        v = q / K;
                        wl_count(L, WL_PSCR, v >= H, mA + v);
                        first = (v < H ? MO::set(hdef, v, 1u << (q % K)) : MO::set(mA, v, 1u << (q % K))) == 0u;
                    }
                    wpush<K>(L, first, v, vscr, &L.qtail, cap, &L.fover, 128u);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                const uint32_t nVs = min(L.qtail, cap);
                __syncthreads();
                // one scan record per (merged vertex p, source j): x = p K + j (a pair listed twice
                // has one); a requested record starts at {+inf, 0 candidates, no slot} and its
                // index is parked in the pair record's third word (read back by the recount), an
                // unrequested one is marked kRsUnreq
                for (uint32_t x = tid; x < nVs * K; x += kSsspBlock) {
                    const uint32_t v = vscr[x / K];
                    const uint32_t j = x % K;
                    const uint32_t m = v < H ? (reinterpret_cast<const uint32_t*>(hdef)[v / MO::kPer] >>
                                                ((v % MO::kPer) * MO::kBits)) & MO::kFull
                                             : MO::get_l2(mA, v);
                    const bool req = (m >> j) & 1u;
                    wl_count(L, WL_PSCR, true, rs + x);
                    {  // {best, candidates | lowest slot << 32}
                        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                        const u64x2 z = {req ? kInfBits : 0ull,
                                         0xFFFFFFFF00000000ull | (req ? 0u : kRsUnreq)};
                        __builtin_nontemporal_store(z, reinterpret_cast<u64x2*>(rs + x));
                    }
                    if (req) {
                        wl_count(L, WL_PREC, true, precw + 4 * ((size_t)v * K + j) + 2);
                        precw[4 * ((size_t)v * K + j) + 2] = x;
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                // one pass over the merged rows: a lane per edge reads the neighbour's K distances
                // (one line) and tests every source of the row's mask
                for (uint32_t base = 0; base < nVs; base += kBChunk) {
                    const uint32_t cnt = min((uint32_t)kBChunk, nVs - base);
                    const uint32_t total = load_chunk<K, false, DIR>(vscr + base, cnt, g, L, D, mA, hdef, false);
                    for (uint32_t e = tid; e < total; e += kSsspBlock) {
                        const int lo = chunk_slot<K>(L, cnt, e);
                        const uint32_t jr = L.rs[lo] + (e - L.off[lo]);
                        const uint32_t m = L.msk[lo];
                        uint32_t u;
                        double wt;
                        adj_load(g, jr, u, wt);
                        unsigned long long du[K];
                        if (u < H) {
#pragma unroll
                            for (int q = 0; q < K; q++) du[q] = D.hd[(size_t)u * K + q];
                        } else {
                            // L1-bypassing 16-B loads of the line (lowered by atomics of other waves)
                            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
                            const u64x2* p = reinterpret_cast<const u64x2*>(D.dist + (size_t)u * K);
#pragma unroll
                            for (int q = 0; q < K / 2; q++) {
                                const u64x2 x = __builtin_nontemporal_load(p + q);
                                du[2 * q] = x.x;
                                du[2 * q + 1] = x.y;
                            }
                        }
                        uint4* const rv = rs + (size_t)(base + (uint32_t)lo) * K;
#pragma unroll
                        for (int q = 0; q < K; q++) {
                            if (((m >> q) & 1u) && __dadd_rn(bits2d(du[q]), wt) == L.val[lo * K + q]) {
                                wl_count(L, WL_PSCR, true, rv + q);
                                atomicMin(reinterpret_cast<unsigned long long*>(rv + q), du[q]);
                                atomicAdd(reinterpret_cast<uint32_t*>(rv + q) + 2, 1u);
                                atomicMin(reinterpret_cast<uint32_t*>(rv + q) + 3, jr);
                            }
                        }
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    __syncthreads();
                }
                if (tid == 0) L.pt[2] += wall_clock64() - tp0;  // merged row scans
                tp0 = wall_clock64();
                // (L1-bypassing reads of the records below: atomics of other waves updated them)
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                // pairs with several candidates: recount at the minimum
                if (tid == 0) L.qtail = 0;
                __syncthreads();
                for (uint32_t xb = 0; xb < nVs * K; xb += kSsspBlock) {
                    const uint32_t x = xb + tid;
                    bool multi = false;
                    uint32_t q = 0;
                    if (x < nVs * K) {
                        const uint32_t c = ld_l2_u32(reinterpret_cast<const uint32_t*>(rs + x) + 2);
                        multi = c > 1u && c != kRsUnreq;
                        wl_count(L, WL_PSCR, multi, rs + x);
                        if (multi) {
                            q = vscr[x / K] * K + x % K;
                            atomicExch(reinterpret_cast<uint32_t*>(rs + x) + 2, 0u);
                            atomicExch(reinterpret_cast<uint32_t*>(rs + x) + 3, 0xFFFFFFFFu);
                        }
                    }
                    wpush<K>(L, multi, q, pnxt, &L.qtail, pcap, &L.fover, 128u);
                }
                __syncthreads();
                const uint32_t nM = min(L.qtail, pcap);
                __syncthreads();
                if (nM > 0) {
                    expand_pairs<K, DIR>(
                        pnxt, nM, g, L,
                        [&](uint32_t q, double& val) { val = bits2d(D.get(q / K, q % K)); },
                        [&](uint32_t q, double dv, uint32_t jr) {
                            uint32_t u;
                            double wt;
                            adj_load(g, jr, u, wt);
                            const unsigned long long du = D.get(u, q % K);
                            uint4* const r = rs + ld_l2_u32(&precw[4 * (size_t)q + 2]);
                            const bool hit = __dadd_rn(bits2d(du), wt) == dv &&
                                             du == ld_l2_u64(reinterpret_cast<const unsigned long long*>(r));
                            wl_count(L, WL_PSCR, hit, r);
                            if (hit) {
                                atomicAdd(reinterpret_cast<uint32_t*>(r) + 2, 1u);
                                atomicMin(reinterpret_cast<uint32_t*>(r) + 3, jr);
                            }
                        });
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                // each requested record stores its pair record (once per pair)
                for (uint32_t x = tid; x < nVs * K; x += kSsspBlock) {
                    const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rs + x));
                    if (r.z == kRsUnreq) continue;
                    const uint32_t q = vscr[x / K] * K + x % K;
                    const uint32_t jr = r.w;
                    const uint32_t c = r.z;
                    wl_count(L, WL_PREC, true, prec + q);
                    if (jr == 0xFFFFFFFFu) {  // unreachable (cannot happen on a connected graph)
                        atomicAdd(&stats[ST_ERRORS], 1ull);
                        prec[q] = make_uint4(L.src[q % K] | 0x40000000u, ept, 0u, 0u);
                    } else {
                        const unsigned long long lb = d2bits(g.aloss[jr]);
                        prec[q] = make_uint4(adj_col(g, jr) | (c > 1 ? 0x80000000u : 0u), ept,
                                             (uint32_t)lb, (uint32_t)(lb >> 32));
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (tid == 0) {
                    L.pt[3] += wall_clock64() - tp0;  // recount + finalize
                    L.rsb = rb + ws.rs_chunk;
                }
                tp0 = wall_clock64();
                __syncthreads();
            }
            __syncthreads();
            if (tid == 0) L.pt[3] += wall_clock64() - tp0;
            tp0 = wall_clock64();
            // the scanned pairs' parents continue as walks
            if (tid == 0) L.qtail = 0;
            __syncthreads();
            for (uint32_t ib = 0; ib < nS; ib += kSsspBlock) {
                const uint32_t i = ib + tid;
                bool p = false;
                uint32_t q = 0;
                const uint32_t qc = i < nS ? fscr[i] : kNoPairS;
                if (qc != kNoPairS) {
                    const uint32_t j = qc % K;
                    // the parent (hint pass or row scan: R's records come from other threads)
                    const uint32_t u = ld_l2_u32(&precw[4 * (size_t)qc]) & 0x3FFFFFFFu;
                    q = u * K + j;
                    p = u != L.src[j];
                }
                wpush<K>(L, p, q, pnxt, &L.qtail, pcap, &L.fover, 128u);
            }
            __syncthreads();
            nF = min(L.qtail, pcap);
            { uint32_t* t = pcur; pcur = pnxt; pnxt = t; }
            plist ^= 1u;
            wkind = kJobWalk;  // later levels start at the scanned pairs' parents (compacted)
            __syncthreads();
            if (tid == 0) L.pt[4] += wall_clock64() - tp0;  // next level
        }
        tick(2);
        if (ws.btrace && tid == 0) ws.btrace[kBTraceWords * (size_t)bidx + 9] = L.tk;

        // ---------------- per-target latency / reliability / hops (shd-topology.c:561-671) ----
        // items (source j, target k) of the whole batch: a job (run_job); row minima in L.rmin
        job_start(kJobEpi);
        run_job(kJobEpi, (uint32_t)A * (uint32_t)nk, ep, (uint32_t)r0, (uint32_t)nk, 0u);
        job_end();
        if ((int)tid < nk) {
            const unsigned long long rm = L.rmin[tid];
            if (out_rowmin) out_rowmin[ws.rowmap ? (int)ws.rowmap[r0 + tid] : r0 + (int)tid] = bits2d(rm);
            atomicMin(&stats[ST_GLOBAL_MIN], rm);  // shd-topology.c:500-511
        }
        __syncthreads();
        tick(3);
        if (ws.btrace && tid == 0) ws.btrace[kBTraceWords * (size_t)bidx + 10] = L.tk;
        {
            // the distance lines this batch lowered from +inf back to +inf: only touched tail
            // vertices (their touched bit in D.pt), not the whole [V][K] block (64 MB at K = 8 per
            // batch); the words are cleared, pending bits included.  Done at the batch's end (its time counts as setup): the next batch's
            // setup waits for these stores; a one-round shard no longer has every slot resetting
            // at its kernel's start.
            // A thread loads one word (16 vertices); the G = K / 2 lanes of a group then reset the
            // group's G words' vertices together, lane p storing the p-th 16 B of each line, so
            // one store instruction writes 64 / G whole lines (one write request per line, not
            // one per 16 B).
            typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
            u64x2* d2 = reinterpret_cast<u64x2*>(D.dist);
            const u64x2 inf2 = {kInfBits, kInfBits};
            constexpr uint32_t G = K / 2;
            const uint32_t part = tid % G, gbase = (tid & 63u) - part;
            unsigned long long nt = 0;
            const uint32_t w0 = H / 32;
            unsigned long long nword = w0 + tid < pw ? ld_l2_u64(&pt2[w0 + tid]) : 0ull;
            for (uint32_t wb = w0; wb < pw; wb += kSsspBlock) {
                const uint32_t wi = wb + tid;
                const unsigned long long word = nword;
                const unsigned long long myw = word & ~kPendBits;  // the touched bits
                rl_count(L, RL_RESET, wi + kSsspBlock < pw, pt2 + wi + kSsspBlock);
                nword = wi + kSsspBlock < pw ? ld_l2_u64(&pt2[wi + kSsspBlock]) : 0ull;
                wl_count(L, WL_TOUCH_CLR, word != 0ull, pt2 + wi);
                if (word) {
                    pt2[wi] = 0ull;
                    nt += (unsigned long long)__popcll(myw);
                }
                if (!__any(myw != 0ull)) continue;
#pragma unroll
                for (uint32_t p = 0; p < G; p++) {
                    unsigned long long w = __shfl(myw, (int)(gbase + p), 64);
                    const uint32_t wv = wi - part + p;
                    while (w) {
                        const uint32_t v = wv * 32u + ((uint32_t)__ffsll((long long)w) - 1u) / 2u;
                        w &= w - 1ull;
                        wl_count(L, WL_RESET, true, d2 + (size_t)v * G + part);
                        __builtin_nontemporal_store(inf2, d2 + (size_t)v * G + part);
                    }
                }
            }
            nt = wave_sum_u64(nt);
            if ((tid & 63) == 0 && nt) atomicAdd(&L.touched, nt);
        }
        tick(0);
        if (ws.btrace && tid == 0) {
            unsigned long long* b = ws.btrace + kBTraceWords * (size_t)bidx;
            b[1] = L.tk;
            b[3] = L.ev[0] - b[3];
            b[4] = L.ev[1] - b[4];
            b[5] = L.ev[2] - b[5];
            b[6] = L.cnt[0] - b[6];
            b[7] = (unsigned long long)nk;
        }
    }
    __syncthreads();
    if (tid == 0) {
        ctr[0] = iter;
        atomicAdd(&stats[ST_RELAX], L.cnt[0]);
        atomicAdd(&stats[ST_T_INIT], L.tm[0]);
        atomicAdd(&stats[ST_T_SSSP], L.tm[1]);
        atomicAdd(&stats[ST_T_PARENT], L.tm[2]);
        atomicAdd(&stats[ST_T_TARGET], L.tm[3]);
        atomicAdd(&stats[ST_T_SPLIT], L.tm[4]);
        atomicAdd(&stats[ST_NEAR_IT], L.ev[0]);
        atomicAdd(&stats[ST_SPLITS], L.ev[1]);
        atomicAdd(&stats[ST_EV0 + 0], L.ev[2]);
        atomicAdd(&stats[ST_EV0 + 3], L.cnt[1]);
        atomicAdd(&stats[ST_EV0 + 1], L.cnt[2]);
        atomicAdd(&stats[ST_EV0 + 6], L.cnt[3]);
        atomicAdd(&stats[ST_EV0 + 2], L.dg[0]);
        atomicAdd(&stats[ST_EV0 + 4], L.dg[1]);
        atomicAdd(&stats[ST_EV0 + 7], L.dg[2]);
        atomicAdd(&stats[ST_TOUCHED], L.touched);
        atomicAdd(&stats[ST_NEAR_IT + 0], 0ull);
        atomicAdd(&stats[ST_OVERSITE], 0ull);
        atomicAdd(&stats[ST_EV0 + 5], 0ull);
        atomicAdd(&stats[ST_EV0 + 5], L.ev[3]);
        for (int i = 0; i < 4; i++) atomicAdd(&stats[ST_PT0 + i], L.pt[1 + i]);
        atomicAdd(&stats[ST_WALK], L.wk[0]);
        for (int i = 0; i < 4; i++) atomicAdd(&stats[ST_WK0 + i], L.wk[1 + i]);
        if (SHD_BATCH_TIME) {
            for (int i = 0; i < 8; i++) atomicAdd(&stats[ST_BT0 + i], L.bt[i]);
            for (int i = 0; i < 4; i++) atomicAdd(&stats[ST_SW0 + i], L.sw[i]);
        }
        if (SHD_BATCH_WRCOUNT) {
            for (int i = 0; i < 16; i++) atomicAdd(&stats[ST_WL0 + i], L.wl[i]);
            for (int i = 0; i < 8; i++) atomicAdd(&stats[ST_RL0 + i], L.rl[i]);
        }
    }
}

__global__ void mark_targets_kernel(uint32_t* __restrict__ adjk, int64_t nadj,
                                    const uint32_t* __restrict__ tbits) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nadj;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t c = adjk[kAdjWords * k];
        const uint32_t v = c & 0x3FFFFFFFu;
        const uint32_t t = (tbits[v >> 5] >> (v & 31u)) & 1u;
        adjk[kAdjWords * k] = (c & ~0x40000000u) | (t << 30);
    }
}

hipError_t launch_mark_targets(uint32_t* adjk, int64_t nadj, const uint32_t* tbits,
                               hipStream_t stream) {
    if (nadj <= 0) return hipSuccess;
    const int64_t g = std::min<int64_t>((nadj + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(mark_targets_kernel, dim3((unsigned)g), dim3(256), 0, stream, adjk, nadj,
                       tbits);
    return hipGetLastError();
}

// Target-aware kappa bound of every vertex (the relaxation's skip test, see phase B).  A pair
// into a non-target tail vertex y is dropped when y's kappa field exceeds the landmark threshold at
// the candidate; kappa0 (the row's smallest w - pi) says "y would relax nothing".  The fixpoint
//   K(x) = min over edges (x, y) of  target(y) ? kap(x, y)
//                                   : max(kap(x, y), K(y) + w (1 - 2e-5) - 1e-9)
// (kap = w - pi(y); K_0 = kappa0) says "y would relax nothing that reaches a target": along a
// parent chain x -> y -> ... -> t the threshold at y is the one at x minus w (plus 1e-5 w of
// margin), so K(x) stays under the threshold of every chain vertex at its final distance (every
// iterate K_k is such a bound; they rise monotonically towards the fixpoint).  Kin == nullptr
// computes K_0.  An edge's kap is static (kfix_kap_kernel, once per graph) and the target test is
// folded into a second array Kt = target ? -inf : K (max(kap, -inf) = kap), so an entry costs one
// random read, Kt[y], instead of three (pi, the target bit and K: 0.52 ms per C4 step).
__global__ void kfix_kap_kernel(const uint32_t* __restrict__ adj, const double* __restrict__ pot,
                                int64_t nadj, double* __restrict__ kap) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nadj;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t y = adj[kAdjWords * k];
        const double w = __hiloint2double((int)adj[kAdjWords * k + 3], (int)adj[kAdjWords * k + 2]);
        const double p = pot[y];
        kap[k] = isfinite(p) ? w - p : -INFINITY;
    }
}

__device__ __forceinline__ double kfix_term(const uint32_t* adj, const double* kap_e,
                                            const double* Ktin, uint32_t k) {
    const double kap = kap_e[k];
    double t = kap;
    if (Ktin) {
        const uint32_t y = adj[kAdjWords * k];
        const double w = __hiloint2double((int)adj[kAdjWords * k + 3], (int)adj[kAdjWords * k + 2]);
        const double ky = Ktin[y] + w * (1.0 - 2e-5) - 1e-9;
        t = ky > kap ? ky : kap;
    }
    return t;
}

__device__ __forceinline__ void kfix_put(double* Kout, double* Ktout, const uint32_t* tbits,
                                         uint32_t x, double m) {
    Kout[x] = m;
    Ktout[x] = ((tbits[x >> 5] >> (x & 31u)) & 1u) ? -INFINITY : m;
}

// A wavefront per segment of a hub row (ids < hs.rows: the long rows of the degree order; a row cut
// in several segments leaves per-segment minima for kfix_multi_kernel), a thread per tail row (a
// wavefront per row left 54 of 64 lanes idle on the C4 tail: 6.2 ms per step; a wavefront per
// whole hub row left the top hub's 250 k entries on one wavefront: 4.4 ms per step).
__global__ void kfix_step_kernel(const uint32_t* __restrict__ rowptr,
                                 const uint32_t* __restrict__ adj, const double* __restrict__ kap_e,
                                 const uint32_t* __restrict__ tbits,
                                 const double* __restrict__ Kin, const double* __restrict__ Ktin,
                                 double* __restrict__ Kout, double* __restrict__ Ktout,
                                 int64_t V, HubSegs hs, double* __restrict__ part,
                                 unsigned int* __restrict__ changed) {
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    bool ch = false;
    for (int64_t s = gt >> 6; s < (int64_t)hs.nseg; s += gs >> 6) {
        const uint2 sg = hs.seg[s];
        const uint32_t x = sg.x, r0 = rowptr[x], r1 = rowptr[x + 1];
        const uint32_t e = min(sg.y + kHubSeg, r1);
        double m = INFINITY;
        for (uint32_t k = sg.y + lane; k < e; k += 64u) {
            const double t = kfix_term(adj, kap_e, Ktin, k);
            m = t < m ? t : m;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double y = __shfl_xor(m, o, 64);
            m = y < m ? y : m;
        }
        if (lane == 0) {
            if (sg.y == r0 && e == r1) {
                ch |= Kin && !(m == Kin[x]);
                kfix_put(Kout, Ktout, tbits, x, m);
            } else {
                part[s] = m;
            }
        }
    }
    for (int64_t x = (int64_t)hs.rows + gt; x < V; x += gs) {
        double m = INFINITY;
        const uint32_t r1 = rowptr[x + 1];
        uint32_t k = rowptr[x];
        // 4 entries at a time: their records and kap, then their neighbours' Kt, all in flight
        for (; k + 4 <= r1; k += 4) {
            double t[4];
#pragma unroll
            for (int i = 0; i < 4; i++) t[i] = kap_e[k + i];
            if (Ktin) {
                uint32_t y[4];
                double w[4], ky[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    y[i] = adj[kAdjWords * (k + i)];
                    w[i] = __hiloint2double((int)adj[kAdjWords * (k + i) + 3],
                                            (int)adj[kAdjWords * (k + i) + 2]);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) ky[i] = Ktin[y[i]];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const double kk = ky[i] + w[i] * (1.0 - 2e-5) - 1e-9;
                    t[i] = kk > t[i] ? kk : t[i];
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) m = t[i] < m ? t[i] : m;
        }
        for (; k < r1; k++) {
            const double t = kfix_term(adj, kap_e, Ktin, k);
            m = t < m ? t : m;
        }
        ch |= Kin && !(m == Kin[x]);
        kfix_put(Kout, Ktout, tbits, (uint32_t)x, m);
    }
    if (__ballot(ch) && lane == 0) atomicOr(changed, 1u);  // one atomic per wave
}

// the hub rows cut in several segments: a wavefront each takes the minimum of its partials
__global__ void kfix_multi_kernel(const double* __restrict__ Kin, double* __restrict__ Kout,
                                  double* __restrict__ Ktout, const uint32_t* __restrict__ tbits,
                                  HubSegs hs, const double* __restrict__ part,
                                  unsigned int* __restrict__ changed) {
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t gs = (int64_t)gridDim.x * blockDim.x;
    bool ch = false;
    for (int64_t i = gt >> 6; i < (int64_t)hs.nmulti; i += gs >> 6) {
        const uint4 mr = hs.multi[i];
        double m = INFINITY;
        for (uint32_t k = lane; k < mr.z; k += 64u) {
            const double t = part[mr.y + k];
            m = t < m ? t : m;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double y = __shfl_xor(m, o, 64);
            m = y < m ? y : m;
        }
        if (lane == 0) {
            ch |= Kin && !(m == Kin[mr.x]);
            kfix_put(Kout, Ktout, tbits, mr.x, m);
        }
    }
    if (__ballot(ch) && lane == 0) atomicOr(changed, 1u);
}

// largest half <= x (NaN: -inf)
__device__ __forceinline__ uint32_t f16_down(double x) {
    if (isnan(x)) return 0xFC00u;
    const _Float16 h = (_Float16)(float)x;
    uint32_t b = (uint32_t)__builtin_bit_cast(unsigned short, h);
    if ((double)(float)h > x) {
        if ((b & 0x7FFFu) == 0u) b = 0x8001u;  // +-0 -> the negative subnormal
        else if (b & 0x8000u) b++;             // negative: larger magnitude
        else b--;                              // positive (or +inf): smaller magnitude
        if ((double)(float)__builtin_bit_cast(_Float16, (unsigned short)b) > x) b = 0xFC00u;
    }
    return b & 0xFFFFu;
}

// the kappa field of every relaxation-copy record := f16 of K(column), rounded down
__global__ void kfix_store_kernel(uint32_t* __restrict__ adjk, int64_t nadj,
                                  const double* __restrict__ K) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nadj;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t y = adjk[kAdjWords * k] & 0x3FFFFFFFu;
        const uint32_t pb = adjk[kAdjWords * k + 1];
        adjk[kAdjWords * k + 1] = (pb & 0xFFFF0000u) | f16_down(K[y]);
    }
}

hipError_t launch_kfix_kap(const uint32_t* adj, const double* pot, int64_t nadj, double* kap,
                           hipStream_t stream) {
    if (nadj <= 0) return hipSuccess;
    const int64_t g = std::min<int64_t>((nadj + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(kfix_kap_kernel, dim3((unsigned)g), dim3(256), 0, stream, adj, pot, nadj, kap);
    return hipGetLastError();
}

hipError_t launch_kfix_step(const uint32_t* rowptr, const uint32_t* adj, const double* kap_e,
                            const uint32_t* tbits, const double* Kin, double* Kout, int64_t V,
                            const HubSegs& hs, double* part, unsigned int* changed,
                            hipStream_t stream) {
    if (V <= 0) return hipSuccess;
    const int64_t g = std::min<int64_t>(std::max<int64_t>((V + 255) / 256, (hs.nseg + 3) / 4), 256 * 32);
    const double* Ktin = Kin ? Kin + V : nullptr;
    hipLaunchKernelGGL(kfix_step_kernel, dim3((unsigned)g), dim3(256), 0, stream, rowptr, adj,
                       kap_e, tbits, Kin, Ktin, Kout, Kout + V, V, hs, part, changed);
    if (hs.nmulti > 0)
        hipLaunchKernelGGL(kfix_multi_kernel, dim3((hs.nmulti + 3) / 4), dim3(256), 0, stream, Kin,
                           Kout, Kout + V, tbits, hs, part, changed);
    return hipGetLastError();
}

// Row order of the relaxation copy for a target set: each row sorted by
// kap'(x, y) = target(y) ? kap(x, y) : max(kap(x, y), K(y) + w (1 - 2e-5) - 1e-9), the same bound
// the pair skip applies per source (a head that relaxes nothing reaching a target sorts past the
// landmark threshold), so the kappa-prefix cut of an expansion stops before such heads.  Keys
// are f32 rounded down: a cut is never too early.
__device__ __forceinline__ float f32_down(double x) {
    if (isnan(x)) return -INFINITY;
    float f = (float)x;
    if ((double)f > x) f = nextafterf(f, -INFINITY);
    return f;
}

__global__ void kprime_key_kernel(const uint32_t* __restrict__ adjk, int64_t nadj,
                                  const double* __restrict__ pot,
                                  const uint32_t* __restrict__ tbits, const double* __restrict__ K,
                                  float* __restrict__ key) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nadj;
         k += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t y = adjk[kAdjWords * k] & 0x3FFFFFFFu;
        const double w = __hiloint2double((int)adjk[kAdjWords * k + 3], (int)adjk[kAdjWords * k + 2]);
        const double p = pot[y];
        double t = isfinite(p) ? w - p : -INFINITY;
        if (!((tbits[y >> 5] >> (y & 31u)) & 1u)) {
            const double ky = K[y] + w * (1.0 - 2e-5) - 1e-9;
            t = ky > t ? ky : t;
        }
        key[k] = f32_down(t);
    }
}

__global__ void kprime_gather_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                     const uint32_t* __restrict__ idx, int64_t nadj) {
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nadj;
         k += (int64_t)gridDim.x * blockDim.x)
        dst[k] = src[idx[k]];
}

__global__ void kprime_probe_kernel(const uint32_t* __restrict__ rowptr,
                                    const float* __restrict__ kap, float* __restrict__ ksum,
                                    float* __restrict__ kap0, int64_t V) {
    for (int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V;
         v += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t b = rowptr[v], n = rowptr[v + 1] - b;
#pragma unroll
        for (int q = 0; q < kKProbes; q++) {
            const uint32_t pq = (1u << q) - 1u;  // 0, 1, 3, 7, 15, 31, 63, 127
            ksum[(size_t)kKProbes * v + q] = pq < n ? kap[b + pq] : INFINITY;
        }
        kap0[v] = n ? kap[b] : INFINITY;
    }
}

// ---- segmented sort of the re-sort keys (replaces a whole-adjacency hipcub segmented radix sort:
// 5.2-5.6 ms at C4 on the first build's critical path, nearly all of it one workgroup per hub row
// sorting that row alone) ----
// The order is hipcub's: ascending by the radix image of the f32 key (-0.0 and +0.0 equal), stable
// (equal keys keep their row positions).  Rows of at most kSegWave entries: one wave per row,
// each lane ranks its entry against the row's others.  Rows up to kSegBlock: one workgroup per
// row, a bitonic sort in LDS of (radix image << 32 | position) -- unique, so the result is the
// stable order; a workgroup takes every G-th row (the long rows are the hubs, at the head of the
// relabelled ids).  Longer rows: their entries (listed once per graph, row by row) are sorted
// together by one device-wide radix sort of (row ordinal << 32 | radix image).
constexpr uint32_t kSegWave = 64;
constexpr uint32_t kSegThreads = 256;

__device__ __forceinline__ uint32_t radix_f32(float f) {
    uint32_t b = __float_as_uint(f);
    b ^= (b & 0x80000000u) ? 0xFFFFFFFFu : 0x80000000u;
    return b == 0x7FFFFFFFu ? 0x80000000u : b;  // -0.0 sorts as +0.0
}

__global__ void __launch_bounds__(kSegThreads)
segsort_wave_kernel(const uint32_t* __restrict__ rowptr, int64_t V, const float* __restrict__ key,
                    float* __restrict__ key_out, uint32_t* __restrict__ idx_out) {
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t nw = ((int64_t)gridDim.x * kSegThreads) >> 6;
    for (int64_t v = ((int64_t)blockIdx.x * kSegThreads + threadIdx.x) >> 6; v < V; v += nw) {
        const uint32_t b = rowptr[v], n = rowptr[v + 1] - b;
        if (n > kSegWave) continue;  // wave-uniform
        float f = 0.0f;
        uint32_t u = 0xFFFFFFFFu;
        if (lane < n) {
            f = key[b + lane];
            u = radix_f32(f);
        }
        uint32_t rank = 0;
        for (uint32_t j = 0; j < n; j++) {
            const uint32_t uj = (uint32_t)__shfl((int)u, (int)j, 64);
            rank += (uj < u || (uj == u && j < lane)) ? 1u : 0u;
        }
        if (lane < n) {
            key_out[b + rank] = f;
            idx_out[b + rank] = b + lane;
        }
    }
}

__global__ void __launch_bounds__(kSegThreads)
segsort_block_kernel(const uint32_t* __restrict__ rowptr, int64_t V, const float* __restrict__ key,
                     float* __restrict__ key_out, uint32_t* __restrict__ idx_out) {
    __shared__ unsigned long long s[kSegBlock];
    __shared__ uint32_t rows[kSegThreads];
    __shared__ uint32_t nrows;
    const uint32_t tid = threadIdx.x;
    const int64_t G = gridDim.x;
    for (int64_t base = 0; base < V; base += G * kSegThreads) {
        // this workgroup's rows base + g + G t (t < 256) that need it
        if (tid == 0) nrows = 0;
        __syncthreads();
        const int64_t v = base + blockIdx.x + G * tid;
        if (v < V) {
            const uint32_t n = rowptr[v + 1] - rowptr[v];
            if (n > kSegWave && n <= kSegBlock) rows[atomicAdd(&nrows, 1u)] = (uint32_t)v;
        }
        __syncthreads();
        const uint32_t nr = nrows;
        __syncthreads();  // every thread has read nrows before the next range resets it
        for (uint32_t i = 0; i < nr; i++) {
            const uint32_t row = rows[i];
            const uint32_t b = rowptr[row], n = rowptr[row + 1] - b;
            uint32_t P = 128;
            while (P < n) P <<= 1;
            for (uint32_t x = tid; x < P; x += kSegThreads)
                s[x] = x < n ? ((unsigned long long)radix_f32(key[b + x]) << 32) | x : ~0ull;
            __syncthreads();
            for (uint32_t k = 2; k <= P; k <<= 1) {
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    for (uint32_t t = tid; t < P / 2; t += kSegThreads) {
                        const uint32_t lo = 2 * t - (t & (j - 1));
                        const uint32_t hi = lo + j;
                        const unsigned long long x = s[lo], y = s[hi];
                        if ((x > y) == ((lo & k) == 0)) {
                            s[lo] = y;
                            s[hi] = x;
                        }
                    }
                    __syncthreads();
                }
            }
            for (uint32_t x = tid; x < n; x += kSegThreads) {
                const uint32_t pos = (uint32_t)s[x];
                key_out[b + x] = key[b + pos];
                idx_out[b + x] = b + pos;
            }
            __syncthreads();
        }
    }
}

__global__ void segsort_gather_kernel(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ row,
                                      int64_t n, const float* __restrict__ key,
                                      unsigned long long* __restrict__ k, uint32_t* __restrict__ val) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = pos[i];
        k[i] = ((unsigned long long)row[i] << 32) | radix_f32(key[p]);
        val[i] = p;
    }
}

// sorted entry i of the long rows goes to the i-th listed position (each row keeps its range)
__global__ void segsort_scatter_kernel(const uint32_t* __restrict__ pos,
                                       const uint32_t* __restrict__ src, int64_t n,
                                       const float* __restrict__ key, float* __restrict__ key_out,
                                       uint32_t* __restrict__ idx_out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t p = pos[i], q = src[i];
        key_out[p] = key[q];
        idx_out[p] = q;
    }
}

hipError_t segsort_big_tmp_bytes(int64_t nitems, int end_bit, size_t* bytes) {
    *bytes = 0;
    if (nitems <= 0) return hipSuccess;
    if (nitems > 0x7FFFFFFF || end_bit < 33 || end_bit > 64) return hipErrorInvalidValue;
    return hipcub::DeviceRadixSort::SortPairs(nullptr, *bytes, (const unsigned long long*)nullptr,
                                              (unsigned long long*)nullptr, (const uint32_t*)nullptr,
                                              (uint32_t*)nullptr, (int)nitems, 0, end_bit,
                                              (hipStream_t)0);
}

hipError_t launch_segsort(const uint32_t* rowptr, int64_t V, int64_t nadj, const float* key,
                          float* key_out, uint32_t* idx_out, const SegBig& big, hipStream_t stream) {
    if (V <= 0 || nadj <= 0) return hipSuccess;
    if (nadj > 0x7FFFFFFF) return hipErrorInvalidValue;
    const int64_t gw = std::min<int64_t>((V * 64 + kSegThreads - 1) / kSegThreads, 256 * 32);
    hipLaunchKernelGGL(segsort_wave_kernel, dim3((unsigned)gw), dim3(kSegThreads), 0, stream, rowptr,
                       V, key, key_out, idx_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t gb = std::min<int64_t>((V + kSegThreads - 1) / kSegThreads, 256 * 8);
    hipLaunchKernelGGL(segsort_block_kernel, dim3((unsigned)gb), dim3(kSegThreads), 0, stream,
                       rowptr, V, key, key_out, idx_out);
    e = hipGetLastError();
    if (e != hipSuccess || big.nitems <= 0) return e;
    if (!big.pos || !big.row || !big.keys || !big.vals || !big.tmp) return hipErrorInvalidValue;
    const int64_t gi = std::min<int64_t>((big.nitems + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(segsort_gather_kernel, dim3((unsigned)gi), dim3(256), 0, stream, big.pos,
                       big.row, big.nitems, key, big.keys, big.vals);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t tb = big.tmp_bytes;
    e = hipcub::DeviceRadixSort::SortPairs(big.tmp, tb, big.keys, big.keys + big.nitems, big.vals,
                                           big.vals + big.nitems, (int)big.nitems, 0, big.end_bit,
                                           stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(segsort_scatter_kernel, dim3((unsigned)gi), dim3(256), 0, stream, big.pos,
                       big.vals + big.nitems, big.nitems, key, key_out, idx_out);
    return hipGetLastError();
}

// the whole-adjacency hipcub sort the kernels above replace (shdtopo_test_segsort's reference)
hipError_t segsort_reference(const uint32_t* rowptr, int64_t V, int64_t nadj, const float* key,
                             const uint32_t* idx_in, float* key_out, uint32_t* idx_out, void* tmp,
                             size_t* tmp_bytes, hipStream_t stream) {
    if (nadj > 0x7FFFFFFF) return hipErrorInvalidValue;
    return hipcub::DeviceSegmentedRadixSort::SortPairs(tmp, *tmp_bytes, key, key_out, idx_in, idx_out,
                                                       (int)nadj, (int)V, rowptr, rowptr + 1, 0, 32,
                                                       stream);
}

hipError_t launch_kprime_resort(uint32_t* adjk, float* kap, float* ksum, float* kap0,
                                const uint32_t* rowptr, int64_t V, int64_t nadj, const double* pot,
                                const uint32_t* tbits, const double* K, const KprimeScratch& sc,
                                hipStream_t stream) {
    if (nadj <= 0 || V <= 0) return hipSuccess;
    if (nadj > 0x7FFFFFFF || !sc.key || !sc.idx || !sc.rec) return hipErrorInvalidValue;
    const int64_t ge = std::min<int64_t>((nadj + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(kprime_key_kernel, dim3((unsigned)ge), dim3(256), 0, stream, adjk, nadj,
                       pot, tbits, K, sc.key);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = launch_segsort(rowptr, V, nadj, sc.key, kap, sc.idx, sc.big, stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(sc.rec, adjk, sizeof(uint4) * (size_t)nadj, hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(kprime_gather_kernel, dim3((unsigned)ge), dim3(256), 0, stream, sc.rec,
                           reinterpret_cast<uint4*>(adjk), sc.idx, nadj);
        e = hipGetLastError();
    }
    if (e == hipSuccess) {
        const int64_t gv = std::min<int64_t>((V + 255) / 256, 256 * 16);
        hipLaunchKernelGGL(kprime_probe_kernel, dim3((unsigned)gv), dim3(256), 0, stream, rowptr,
                           kap, ksum, kap0, V);
        e = hipGetLastError();
    }
    return e;
}

hipError_t launch_kfix_store(uint32_t* adjk, int64_t nadj, const double* K, hipStream_t stream) {
    if (nadj <= 0) return hipSuccess;
    const int64_t g = std::min<int64_t>((nadj + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(kfix_store_kernel, dim3((unsigned)g), dim3(256), 0, stream, adjk, nadj, K);
    return hipGetLastError();
}

SsspLdsPlan sssp_batch_lds_plan(int K, int64_t hub_limit, uint32_t par_hubs, int64_t V) {
    auto bytes = [&](uint32_t H, uint32_t P) -> size_t {
        switch (K) {
            case 2: return blayout<2>(H, P).bytes;
            case 4: return blayout<4>(H, P).bytes;
            case 8: return blayout<8>(H, P).bytes;
            case 16: return blayout<16>(H, P).bytes;
        }
        return (size_t)-1;
    };
    SsspLdsPlan p;
    if (bytes(0, 0) == (size_t)-1) return p;
    int64_t H = 0;
    while (true) {  // largest H (multiple of 16) whose layout fits with P = min(par_hubs, H)
        const int64_t h2 = H + 16;
        const uint32_t P2 = (uint32_t)std::min<int64_t>(par_hubs, h2);
        if (bytes((uint32_t)h2, P2) > kBMaxLds) break;
        H = h2;
    }
    if (hub_limit >= 0 && hub_limit < H) H = hub_limit;
    if (H > V) H = V;
    p.H = (uint32_t)H;
    p.P = (uint32_t)std::min<int64_t>(par_hubs, H);
    p.bytes = bytes(p.H, p.P);
    return p;
}

template <int K>
static hipError_t launch_batch_k(const DevCSR& g, const SlotWs& ws, const uint32_t* d_sources,
                                 const double* d_srcsh, int nsrc, int kf, const uint32_t* d_targets,
                                 int A, double delta, const SsspLdsPlan& plan, uint32_t iter_guard,
                                 double2* out_lr, uint16_t* out_hops, double* out_rowmin,
                                 unsigned long long* d_stats, hipStream_t stream) {
    if (kf < 1 || kf > K) return hipErrorInvalidValue;
    // (a layout's batches are checked on the host: each within 1..K positions, covering [0, nsrc))
    const int nb = ws.bstart ? ws.nbat : (nsrc + kf - 1) / kf;
    const int grid = ws.slots < nb ? ws.slots : nb;
    if (grid < 1) return hipSuccess;
    if ((int64_t)plan.H > g.V || plan.P > plan.H || plan.bytes > kBMaxLds ||
        blayout<K>(plan.H, plan.P).bytes != plan.bytes || ws.K != K)
        return hipErrorInvalidValue;
    auto* kern = g.directed ? sssp_batch_kernel<K, true> : sssp_batch_kernel<K, false>;
    {  // per device (multi-GPU builds launch on several): set before every launch
        hipError_t e = hipFuncSetAttribute((const void*)kern,
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)kBMaxLds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kSsspBlock), plan.bytes, stream, g,
                       ws, d_sources, d_srcsh, nsrc, kf, d_targets, A, delta, plan.H, plan.P, iter_guard,
                       out_lr, out_hops, out_rowmin, d_stats);
    return hipGetLastError();
}

hipError_t launch_sssp_batch(int K, const DevCSR& g, const SlotWs& ws, const uint32_t* d_sources,
                             const double* d_srcsh, int nsrc, int kf, const uint32_t* d_targets,
                             int A, double delta, const SsspLdsPlan& plan, uint32_t iter_guard,
                             double2* out_lr, uint16_t* out_hops, double* out_rowmin,
                             unsigned long long* d_stats, hipStream_t stream) {
    switch (K) {
        case 2: return launch_batch_k<2>(g, ws, d_sources, d_srcsh, nsrc, kf, d_targets, A, delta, plan, iter_guard, out_lr, out_hops, out_rowmin, d_stats, stream);
        case 4: return launch_batch_k<4>(g, ws, d_sources, d_srcsh, nsrc, kf, d_targets, A, delta, plan, iter_guard, out_lr, out_hops, out_rowmin, d_stats, stream);
        case 8: return launch_batch_k<8>(g, ws, d_sources, d_srcsh, nsrc, kf, d_targets, A, delta, plan, iter_guard, out_lr, out_hops, out_rowmin, d_stats, stream);
        case 16: return launch_batch_k<16>(g, ws, d_sources, d_srcsh, nsrc, kf, d_targets, A, delta, plan, iter_guard, out_lr, out_hops, out_rowmin, d_stats, stream);
    }
    return hipErrorInvalidValue;
}

hipError_t preload_batch_module() {
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, (const void*)sssp_batch_kernel<8, false>);
}

// The first hipcub sort of a kind in a process spends ~12 ms of host time before its first
// kernel (measured by tools/sort_warm_probe.cpp for the segmented radix sort: 11.9 ms, then
// 0.016 ms per call).  The target preparation's re-sort of the long rows is the first one a build
// runs, so the background init sorts a few keys of that kind first.
hipError_t preload_kprime_sort(hipStream_t stream) {
    constexpr int kN = 256;
    uint8_t* buf = nullptr;
    size_t tb = 0;
    hipError_t e = segsort_big_tmp_bytes(kN, 40, &tb);
    if (e == hipSuccess) e = hipMalloc(&buf, 2 * 12 * (size_t)kN + tb);
    if (e != hipSuccess) return e;
    unsigned long long* k = reinterpret_cast<unsigned long long*>(buf);
    uint32_t* v = reinterpret_cast<uint32_t*>(buf + 16 * (size_t)kN);
    e = hipMemsetAsync(buf, 0, 2 * 12 * (size_t)kN, stream);
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(buf + 24 * (size_t)kN, tb, k, k + kN, v, v + kN, kN,
                                               0, 40, stream);
    const hipError_t s = hipStreamSynchronize(stream);
    (void)hipFree(buf);
    return e != hipSuccess ? e : s;
}

}  // namespace shdtopo
