// topo_replay.hip -- exact igraph-0.7 Dijkstra replay for gfx950: one wavefront per source runs
// the reference's heap algorithm operation for operation, so that parents on equal-distance ties
// (igraph's pop order among equal keys) come out exactly as the reference's.
//
// Why.  The batched delta-stepping kernel (topo_sssp_batch.hip) computes every distance bit-exact
// and every parent that has a single candidate.  Where a vertex v has several candidates u with
// the same minimal d[u] (integer latencies: common), igraph's parent is the candidate popped
// first from its two-way heap, and that order is a sequential heap history.  The
// batch kernel flags every such row (memo bit 31 -> rowflag); this kernel recomputes exactly
// those rows (and every row of a directed topology, where the batch kernel does not run).
//
// What is replayed (igraph 0.7.1, restated in oracle/oracle.c:146-305 and SURVEY.md A.3):
//   * igraph_get_shortest_paths_dijkstra (structural_properties.c): dist = -1, push(src, 0);
//     while (size > 0 && to_reach > 0): pop max; to_reach -= is_target; relax the incident
//     edges in igraph_incident order: dist < 0 -> dist = alt, parent = e, push(-alt);
//     alt < dist (strict) -> dist = alt, parent = e, modify(-alt);
//   * igraph_2wheap_t (indheap.c): max-heap on -dist, PARENT(x) = (x+1)/2-1;
//     shift_up swaps while data[x] >= data[parent]; delete_max swaps root and last, pops, sinks;
//     sink takes the left child if right == size || data[L] >= data[R], swaps if
//     data[head] < data[child]; modify = set, sink (a no-op for a larger key), shift_up;
//   * the per-target helper shd-topology.c:561-671 for the epilogue (reliability product in
//     path order from the source, latency = left-to-right sum of the igraph_get_eid edges).
// Incidence order (type_indexededgelist.c): for an undirected graph out-list (neighbours <= x)
// then in-list (neighbours >= x), i.e. ascending neighbour id (original numbering) with self
// loops in the middle (they never relax); directed, mode OUT: out-neighbours ascending.  The
// host builds rows in that order (relabelled ids, parallel edges merged: see below).
//
// Parallel edges.  igraph relaxes them one after another; for a group of parallel edges the
// heap ends in the same state as one relaxation with the group's minimum latency (a shift-up
// from a position on the ancestor chain stops where the largest key stops, keys being monotone
// along the chain), so the host merges them.  The epilogue uses the igraph_get_eid edge of each
// hop (lowest edge id, as the oracle) for latency and loss.
//
// Wavefront mapping.  Heap operations are inherently sequential; the 64 lanes make each one
// short instead: a sink loads the 62-node subtree five levels below the current node in one
// round trip (positions of a level are contiguous: a few cache lines) and walks it in
// registers; a shift-up loads the whole ancestor chain (<= 20 lanes) in one round trip and
// finds its stop by a ballot; the relaxation of a row takes 64 edges per step.  The top
// kRpLdsLevels levels of the heap live in LDS (the positions every sink starts from).
//
// Landmark skip.  Half the relaxations go to vertices already popped (each undirected edge is
// relaxed from both ends) and change nothing, yet each reads a random 16-B vertex record.  The
// row entry carries pi(t) = d(h0, t) (f32 rounded up; h0 = the top hub, relabelled vertex 0);
// once h0 is popped, d(h0) + pi(t) < du (with a 1e-6 relative margin for the rounding of the
// sums) proves t popped, and its record is not read: on C4-int 31-46 % of the relaxations.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "topo_dev_common.h"

namespace shdtopo {

namespace {

using namespace dev;

#ifndef SHD_RP_LDS_LEVELS
#define SHD_RP_LDS_LEVELS 9       // f64 keys: 511 x 12 B in LDS per wavefront
#endif
#ifndef SHD_RP_LDS_LEVELS_INT
#define SHD_RP_LDS_LEVELS_INT 9   // u32 keys: 511 x 8 B (10 levels, 8 KiB, lose occupancy: +28 %)
#endif
#ifndef SHD_RP_LINES
#define SHD_RP_LINES 0  // profiling build: count the 64-B lines each part of the replay touches
#endif
#ifndef SHD_RP_TIME
#define SHD_RP_TIME 0  // profiling build: wall time per part of a pop (sink, row + record loads,
                       // heap operations of the relaxation, init + epilogue)
#endif
#if SHD_RP_TIME
#define RP_TICK(i) do { const unsigned long long t_ = wall_clock64(); tph[i] += t_ - tlast; tlast = t_; } while (0)
#else
#define RP_TICK(i) do { } while (0)
#endif
#if SHD_RP_TIME  // sink sub-phases: LDS walk, HBM rounds, moves (nl[8..10], clock in nl[12])
#define RP_STICK(i) do { const unsigned long long t_ = wall_clock64(); H.nl[8 + (i)] += t_ - H.nl[12]; H.nl[12] = t_; } while (0)
#else
#define RP_STICK(i) do { } while (0)
#endif
constexpr int kRpLA = 5;  // LDS walk of the sink: heap levels per LDS round (62 nodes)
#ifndef SHD_RP_HL
#define SHD_RP_HL 5  // levels per HBM round of the path-first sink (6: two nodes per lane)
#endif
constexpr int kHL = SHD_RP_HL;
constexpr int kHNodes = (2 << kHL) - 2;
static_assert(kHL >= 1 && kHNodes <= 128, "at most two nodes per lane");

__device__ __forceinline__ uint32_t rl_u32(uint32_t x, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}
__device__ __forceinline__ double rl_f64(double x, int l) {
    const unsigned long long b = d2bits(x);
    const uint32_t lo = rl_u32((uint32_t)b, l), hi = rl_u32((uint32_t)(b >> 32), l);
    return bits2d(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t uni_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ double uni_f64(double x) { return rl_f64(x, 0); }

// Heap keys.  igraph's two-way heap holds data = -dist (a max-heap).  Two exact encodings:
//   * f64 (any latencies): key = -dist, 16-B HBM nodes {f64 key, u32 vertex, pad};
//   * u32 (option replay_int_keys, when every latency is an integer and V x max latency fits in
//     u32 -- upload_replay checks it): dist is an integer < 2^32 - 1, every f64 sum the reference
//     forms is exact, and key = ~dist orders as -dist does (~ reverses the u32 order), so every
//     comparison -- ties included -- is the f64 one.  8-B nodes {u32 key, u32 vertex}: a sink
//     round's 62-node subtree is half the lines, and the readlane walks move one word per key.
// Vertex records stay 16 B {dist, pad | f64 dist, u32 parent slot, u32 heap position}.
template <bool I> struct RpKey;
template <> struct RpKey<false> {
    using T = double;
    using Node = uint4;
    static constexpr int kLevels = SHD_RP_LDS_LEVELS;
    static constexpr unsigned long long kUnreached = 0xBFF0000000000000ull;  // dist = -1.0
    __device__ static T lo() { return -INFINITY; }
    __device__ static T hi() { return INFINITY; }
    __device__ static T rl(T x, int l) { return rl_f64(x, l); }
    __device__ static T uni(T x) { return uni_f64(x); }
    __device__ static Node pack(T k, uint32_t v) {
        const unsigned long long b = d2bits(k);
        return make_uint4((uint32_t)b, (uint32_t)(b >> 32), v, 0u);
    }
    __device__ static void unpack(const Node& q, T& k, uint32_t& v) {
        k = __hiloint2double((int)q.y, (int)q.x);
        v = q.z;
    }
    __device__ static T dist(const uint4& x) { return __hiloint2double((int)x.y, (int)x.x); }
    __device__ static bool reached(T d) { return d >= 0.0; }
    __device__ static T key_of(T d) { return -d; }
    __device__ static T dist_of_key(T k) { return -k; }
    __device__ static T src_key() { return 0.0; }
    __device__ static double f64(T d) { return d; }
    __device__ static T add(T d, double w) { return __dadd_rn(d, w); }
    __device__ static uint3 rec(T d, uint32_t j) {
        const unsigned long long b = d2bits(d);
        return make_uint3((uint32_t)b, (uint32_t)(b >> 32), j);
    }
    __device__ static void set_dist(uint4* r, T d) { *reinterpret_cast<double*>(r) = d; }
};
template <> struct RpKey<true> {
    using T = uint32_t;
    using Node = uint2;
    static constexpr int kLevels = SHD_RP_LDS_LEVELS_INT;
    static constexpr unsigned long long kUnreached = ~0ull;  // dist word = 0xFFFFFFFF
    __device__ static T lo() { return 0u; }
    __device__ static T hi() { return 0xFFFFFFFFu; }
    __device__ static T rl(T x, int l) { return rl_u32(x, l); }
    __device__ static T uni(T x) { return uni_u32(x); }
    __device__ static Node pack(T k, uint32_t v) { return make_uint2(k, v); }
    __device__ static void unpack(const Node& q, T& k, uint32_t& v) {
        k = q.x;
        v = q.y;
    }
    __device__ static T dist(const uint4& x) { return x.x; }
    __device__ static bool reached(T d) { return d != 0xFFFFFFFFu; }
    __device__ static T key_of(T d) { return ~d; }
    __device__ static T dist_of_key(T k) { return ~k; }
    __device__ static T src_key() { return ~0u; }
    __device__ static double f64(T d) { return (double)d; }
    // w is an integer-valued f64 and du + w < 2^32 - 1 (the host's bound): exact
    __device__ static T add(T d, double w) { return d + (uint32_t)w; }
    __device__ static uint3 rec(T d, uint32_t j) { return make_uint3(d, 0xFFFFFFFFu, j); }
    __device__ static void set_dist(uint4* r, T d) { *reinterpret_cast<uint32_t*>(r) = d; }
};

// 64-B lines touched by one wave-wide access (active lanes, addresses ascending in lane order
// for the heap's subtree / chain accesses; a random gather counts one line per lane).
enum { RPL_SINK_LD, RPL_SINK_ST, RPL_SHIFT_LD, RPL_SHIFT_ST, RPL_RELAX_LD, RPL_RELAX_ST };
__device__ __forceinline__ void rp_lines(unsigned long long* nl, int cat, bool act, const void* a) {
#if SHD_RP_LINES
    const unsigned long long line = (unsigned long long)a >> 6;
    const unsigned long long am = __ballot(act);
    const int lane = (int)__lane_id();
    const unsigned long long prev = __shfl_up(line, 1);
    const bool dup = lane > 0 && ((am >> (lane - 1)) & 1ull) && prev == line;
    const unsigned long long nm = __ballot(act && !dup);
    if (lane == __ffsll((long long)am) - 1) nl[cat] += (unsigned long long)__popcll(nm);
#else
    (void)nl; (void)cat; (void)act; (void)a;
#endif
}

// The heap's top levels (positions < kT) of this workgroup's (= wavefront's) source, in LDS.
// File-scope __shared__ reached only through these accessors: every access is a ds_read /
// ds_write (a generic pointer let the compiler merge the LDS and HBM branches of a node access
// into flat loads, which wait on both counters and serialised the sink behind outstanding HBM
// loads: -4 to -7 %).  Each kernel instantiation references (and is allocated) one pair.
constexpr uint32_t kRpTF = (1u << SHD_RP_LDS_LEVELS) - 1u;
constexpr uint32_t kRpTI = (1u << SHD_RP_LDS_LEVELS_INT) - 1u;
__shared__ double rp_sk[kRpTF];
__shared__ uint32_t rp_sv[kRpTF];
__shared__ uint32_t rp_ik[kRpTI];
__shared__ uint32_t rp_iv[kRpTI];
template <bool I>
__device__ __forceinline__ typename RpKey<I>::T lds_k(uint32_t p) {
    if constexpr (I) return rp_ik[p];
    else return rp_sk[p];
}
template <bool I>
__device__ __forceinline__ uint32_t lds_v(uint32_t p) {
    if constexpr (I) return rp_iv[p];
    else return rp_sv[p];
}
template <bool I>
__device__ __forceinline__ void lds_put(uint32_t p, typename RpKey<I>::T k, uint32_t v) {
    if constexpr (I) {
        rp_ik[p] = k;
        rp_iv[p] = v;
    } else {
        rp_sk[p] = k;
        rp_sv[p] = v;
    }
}

// The heap of one source: keys (igraph's data = -dist, encoded per RpKey) and vertices,
// positions < kT in LDS, the rest as nodes in this slot's HBM (one line per node access); the
// position of a queued vertex lives in its 16-B vertex record (one line per relaxation target).
// For a vertex in the LDS levels the record only says so (some position < kT): moves inside
// the LDS levels (half of every sink path) store no position -- each would be a 4-B write to a
// random line -- and a modify of such a vertex finds it by a wave-wide search of the LDS vertex
// array (rp_lds_find).
template <bool I>
struct RpHeap {
    using K = RpKey<I>;
    using T = typename K::T;
    static constexpr uint32_t kT = (1u << K::kLevels) - 1u;
    typename K::Node* gn;
    uint4* vr;
    unsigned long long* nl;
    uint32_t stdPos, stdBase;
    // Physical node of HBM position p (positions below stdPos = kT live in LDS).  (Round 5 also
    // had a banded layout -- a sink round's subtree in one contiguous block -- measured slower and
    // removed in round 6: DESIGN.md 4.)
    __device__ __forceinline__ uint32_t phys(uint32_t p) const { return p - stdPos + stdBase; }
    __device__ __forceinline__ void node(uint32_t p, T& k, uint32_t& v, int cat) const {
        if (p < kT) {
            k = lds_k<I>(p);
            v = lds_v<I>(p);
        } else {
            const uint32_t x = phys(p);
            rp_lines(nl, cat, true, gn + x);
            K::unpack(gn[x], k, v);
        }
    }
    // node (k, v) to position p; its vertex record's position is stored only when `pos` (the
    // element crossed into or out of the LDS levels, moved inside the HBM levels, or is new)
    __device__ __forceinline__ void put(uint32_t p, T k, uint32_t v, int cat, bool pos = true) const {
        rp_lines(nl, cat, pos, vr + 4 * (size_t)__lane_id() + v);  // random: one line each
        if (p < kT) {
            lds_put<I>(p, k, v);
        } else {
            const uint32_t x = phys(p);
            rp_lines(nl, cat, true, gn + x);
            gn[x] = K::pack(k, v);
        }
        if (pos) reinterpret_cast<uint32_t*>(vr + v)[3] = p;
    }
};

// Heap position of this lane's node in the subtree kRpLA levels below `head` (BFS order).
__device__ __forceinline__ uint32_t rp_sub_pos(uint32_t head, int lane) {
    const uint32_t rr = (uint32_t)lane + 2u;  // BFS index + 1 of this lane's subtree node
    const int dl = 31 - __clz(rr);            // its depth below the hole (1..kRpLA)
    return ((head + 1u) << dl) - 1u + (rr - (1u << dl));
}

// Position of vertex t among the heap's LDS levels (positions < min(size, kT)): every lane
// checks its share of the LDS vertex array, one ballot.  ~0u: not there (cannot happen for a
// vertex whose record says it is).
template <bool I>
__device__ __forceinline__ uint32_t rp_lds_find(uint32_t t, uint32_t size, int lane) {
    constexpr uint32_t kT = RpHeap<I>::kT;
    const uint32_t n = size < kT ? size : kT;
    uint32_t found = 0xFFFFFFFFu;
    for (uint32_t b = 0; b < n; b += 64u) {
        const uint32_t p = b + (uint32_t)lane;
        const unsigned long long m = __ballot(p < n && lds_v<I>(p) == t);
        if (m) {
            found = b + (uint32_t)(__ffsll((long long)m) - 1);
            break;
        }
    }
    return found;
}

// One sink round's path of larger children, lane-parallel: lane i holds node rr = i + 2 of the
// subtree below the round's head (BFS, head = 1; `valid`: the node exists, i.e. its position is
// below the heap size).  igraph_2wheap_sink goes left when data[L] >= data[R] (or R does not
// exist): every node compares itself with its sibling (one shuffle) -- the winners form one
// ballot -- and a node is on the path iff it and all its ancestors below the head won (bit tests
// of that ballot).  A second ballot is the path, one node per depth; path lanes np .. np + m - 1
// receive node (position, key, vertex) of depth 1 .. m by one shuffle each.  No readlane chain:
// a few dozen VALU and three ballots instead of la dependent readlane steps.  Returns m (levels
// taken: < la when the path ends inside the round); *cur becomes the deepest path node.
template <bool I>
__device__ __forceinline__ int rp_round_path(uint32_t& cur, int lane, bool valid,
                                             typename RpKey<I>::T k, uint32_t v, uint32_t p,
                                             int np, uint32_t& pp, typename RpKey<I>::T& pk,
                                             uint32_t& pv) {
    using T = typename RpKey<I>::T;
    const uint32_t rr = (uint32_t)lane + 2u;
    const T ks = __shfl_xor(k, 1, 64);
    const bool vs = __shfl_xor(valid ? 1 : 0, 1, 64) != 0;
    // left (rr even) wins if it exists and (no right sibling or k_L >= k_R); right wins if both
    // exist and !(k_L >= k_R)
    const bool win = (rr & 1u) == 0u ? (valid && (!vs || k >= ks)) : (valid && vs && !(ks >= k));
    const unsigned long long W = __ballot(win);
    bool on = win;
#pragma unroll
    for (int t = 1; t < kRpLA; t++) {
        const uint32_t a = rr >> t;  // ancestor at t levels up (a >= 2: below the head)
        if (a >= 2u) on = on && ((W >> (a - 2u)) & 1ull);
    }
    const unsigned long long P = __ballot(on);
    const int m = __popcll(P);
    // lane np + d - 1 takes the path node of depth d (lanes rr in [2^d, 2^(d+1)))
    const int d = lane - np + 1;
    int src = 0;
    if (d >= 1 && d <= m) {
        const unsigned long long rng = ((2ull << ((1u << d) - 1u)) - 1ull) << ((1u << d) - 2u);
        src = __ffsll((long long)(P & rng)) - 1;
    }
    const T ksrc = __shfl(k, src, 64);
    const uint32_t vsrc = __shfl(v, src, 64), psrc = __shfl(p, src, 64);
    if (d >= 1 && d <= m) {
        pp = psrc;
        pk = ksrc;
        pv = vsrc;
    }
    if (m > 0) cur = rl_u32(p, 63 - __clzll((long long)P));
    return m;
}

// igraph_2wheap_delete_max's sink of x = the last element from the root (a hole) in a heap of
// `size` (after the removal): igraph_2wheap_sink takes the left child if right == size or
// data[L] >= data[R] and swaps while data[head] < data[child].  The path of larger children does
// not depend on x, so it is found first: the LDS levels by lane-parallel LDS reads while x's
// load is in flight, then the HBM levels kHL per round trip.  x stops at the first path node it
// is not smaller than; the path nodes above the stop move up one level, in parallel (lane i
// holds path node i).  (kx, vx): x in lane 63, loaded by the caller.
template <bool I>
__device__ __forceinline__ void rp_pop_sink(const RpHeap<I>& H, uint32_t size, int lane,
                                            typename RpKey<I>::T kx, uint32_t vx) {
    using K = RpKey<I>;
    using T = typename K::T;
    constexpr uint32_t kT = RpHeap<I>::kT;
#if SHD_RP_TIME
    H.nl[12] = wall_clock64();
#endif
    uint32_t pp = 0, pv = 0;  // this lane's path node: position, vertex, key
    T pk = K::hi();
    int np = 0;
    uint32_t cur = 0;
    bool bottom = false;
    // LDS levels, kRpLA per round: every lane reads its subtree node (one LDS round trip), the
    // path is walked with readlanes
    for (;;) {
        const int dcur = 31 - __clz(cur + 1u);   // level of cur
        const int nlds = K::kLevels - 1 - dcur;  // LDS levels below it
        if (nlds <= 0) break;
        const int la = nlds < kRpLA ? nlds : kRpLA;
        const uint32_t p = rp_sub_pos(cur, lane);
        T k = K::lo();
        uint32_t v = 0;
        const bool valid = lane < (2 << la) - 2 && p < size;
        if (valid) {
            k = lds_k<I>(p);
            v = lds_v<I>(p);
        }
        {
            const int m = rp_round_path<I>(cur, lane, valid, k, v, p, np, pp, pk, pv);
            np += m;
            if (m < la) {
                bottom = true;
                break;
            }
            continue;
        }
        uint32_t q = 0;
        for (int s = 0; s < la; ++s) {
            const uint32_t L = 2u * cur + 1u;
            if (L >= size) {
                bottom = true;
                break;
            }
            const int li = (int)(2u * q);  // BFS index of the left child
            const T kL = K::rl(k, li);
            int ci = li;
            uint32_t c = L;
            T kc = kL;
            if (L + 1u < size) {
                const T kR = K::rl(k, li + 1);
                if (!(kL >= kR)) {
                    ci = li + 1;
                    c = L + 1u;
                    kc = kR;
                }
            }
            const uint32_t vc = rl_u32(v, ci);
            if (lane == np) {
                pp = c;
                pk = kc;
                pv = vc;
            }
            cur = c;
            np++;
            q = (uint32_t)ci + 1u;
        }
        if (bottom) break;
    }
    RP_STICK(0);
    T xk = K::lo();
    uint32_t xv = 0;
    bool havex = false;
    int stop = -1;  // first path index x is not smaller than
    while (!bottom) {
#if SHD_RP_TIME
        H.nl[6]++;  // HBM sink rounds
#endif
        const uint32_t p = rp_sub_pos(cur, lane);
        T k = K::lo(), k2 = K::lo();
        uint32_t v = 0, v2 = 0;
        if (lane < kHNodes && p < size)
            H.node(p, k, v, RPL_SINK_LD);
        if (kHNodes > 64) {  // BFS nodes 64.. in a second register
            const uint32_t p2 = rp_sub_pos(cur, lane + 64);
            if (lane + 64 < kHNodes && p2 < size)
                H.node(p2, k2, v2, RPL_SINK_LD);
        }
        if (!havex) {
            xk = K::rl(kx, 63);
            xv = rl_u32(vx, 63);
            havex = true;
            const unsigned long long sm = __ballot(lane < np && !(xk < pk));
            if (sm) {
                stop = __ffsll((long long)sm) - 1;
                break;
            }
        }
        if (kHNodes <= 64) {
            // the round's path at once; x stops at the first of its nodes it is not smaller than
            const bool valid = lane < kHNodes && p < size;
            const int np0 = np;
            const int m = rp_round_path<I>(cur, lane, valid, k, v, p, np, pp, pk, pv);
            np += m;
            const unsigned long long sm = __ballot(lane >= np0 && lane < np && !(xk < pk));
            if (sm) {
                stop = __ffsll((long long)sm) - 1;
                break;
            }
            if (m < kHL) bottom = true;
            continue;
        }
        uint32_t q = 0;
#pragma unroll
        for (int s = 0; s < kHL; ++s) {
            const uint32_t L = 2u * cur + 1u;
            if (L >= size) {
                bottom = true;
                break;
            }
            const int li = (int)(2u * q);  // BFS index of the left child (2q+1 - 1)
            const T kL = li < 64 ? K::rl(k, li) : K::rl(k2, li - 64);
            int ci = li;
            uint32_t c = L;
            T kc = kL;
            if (L + 1u < size) {
                const T kR = li + 1 < 64 ? K::rl(k, li + 1) : K::rl(k2, li + 1 - 64);
                if (!(kL >= kR)) {
                    ci = li + 1;
                    c = L + 1u;
                    kc = kR;
                }
            }
            if (!(xk < kc)) {
                stop = np;
                break;
            }
            const uint32_t vc = ci < 64 ? rl_u32(v, ci) : rl_u32(v2, ci - 64);
            if (lane == np) {
                pp = c;
                pk = kc;
                pv = vc;
            }
            cur = c;
            np++;
            q = (uint32_t)ci + 1u;
        }
        if (stop >= 0) break;
    }
    if (!havex) {
        xk = K::rl(kx, 63);
        xv = rl_u32(vx, 63);
        const unsigned long long sm = __ballot(lane < np && !(xk < pk));
        stop = sm ? __ffsll((long long)sm) - 1 : np;
    } else if (stop < 0) {
        stop = np;
    }
    RP_STICK(1);
    const uint32_t up = __shfl_up(pp, 1);  // the parent's position (path node lane - 1)
    if (lane < stop) H.put(lane == 0 ? 0u : up, pk, pv, RPL_SINK_ST, pp >= kT);
    if (lane == 0) {
        const uint32_t xp = stop == 0 ? 0u : rl_u32(pp, stop - 1);
        H.put(xp, xk, xv, RPL_SINK_ST, xp >= kT || size >= kT);  // x came from position size
    }
    RP_STICK(2);
}

// igraph_2wheap_shift_up of element (xk, xv) from position `pos` (a hole).  Returns the number f
// of ancestors moved down one level; lane i < f holds the moved vertex (mv) and its new position.
// Most shift-ups stop below the parent: it is read first (one node), the whole chain only when x
// rises past it.  check = false: the caller knows x rises past the parent.
template <bool I>
__device__ __forceinline__ int rp_shift_up(const RpHeap<I>& H, uint32_t pos,
                                           typename RpKey<I>::T xk, uint32_t xv, int lane,
                                           uint32_t& mv, uint32_t& mp, bool fresh,
                                           bool check = true) {
    using K = RpKey<I>;
    using T = typename K::T;
    constexpr uint32_t kT = RpHeap<I>::kT;
    if (check && pos > 0) {
        T k0;
        uint32_t v0;
        H.node((pos - 1u) >> 1, k0, v0, RPL_SHIFT_LD);
        if (xk < K::uni(k0)) {  // data[x] < data[parent]: stays (a pushed vertex is new)
            if (lane == 0) H.put(pos, xk, xv, RPL_SHIFT_ST, fresh);
            return 0;
        }
    }
    const uint32_t depth = (uint32_t)(31 - __clz(pos + 1u));  // ancestors of pos
    const bool valid = (uint32_t)lane < depth;
    const uint32_t sh = valid ? (uint32_t)lane + 1u : 0u;
    const uint32_t a = ((pos + 1u) >> sh) - 1u;
    T ak = K::hi();
    uint32_t av = 0;
    if (valid) H.node(a, ak, av, RPL_SHIFT_LD);
    // x rises past every ancestor with key <= x and stops below the first one with key > x
    const unsigned long long stopm = __ballot(valid && xk < ak);
    const int f = stopm ? __ffsll((long long)stopm) - 1 : (int)depth;
    const uint32_t c = lane == 0 ? pos : (valid ? ((pos + 1u) >> (uint32_t)lane) - 1u : 0u);
    if (lane < f) H.put(c, ak, av, RPL_SHIFT_ST, c >= kT);  // ancestors move down to c
    const uint32_t fp = f == 0 ? pos : ((pos + 1u) >> (uint32_t)f) - 1u;
    if (lane == 0) H.put(fp, xk, xv, RPL_SHIFT_ST, fresh || (f > 0 && (fp >= kT || pos >= kT)));
    mv = av;
    mp = c;
    return f;
}

__device__ __forceinline__ uint32_t vr_par(const uint4* vr, uint32_t v) { return vr[v].z; }

#ifndef SHD_RP_WAVES_EU
#define SHD_RP_WAVES_EU 4  // minimum waves per SIMD the register allocation must allow
#endif
template <bool I>
__global__ void __launch_bounds__(64, SHD_RP_WAVES_EU)
heap_replay_kernel(ReplayCSR g, ReplayWs ws, const uint32_t* __restrict__ sources,
                   const uint32_t* __restrict__ rows, int nrows,
                   const uint32_t* __restrict__ targets, int A, int full, double2* out_lr,
                   uint16_t* out_hops, double* out_rowmin, unsigned long long* stats,
                   double* dbg_dist, int32_t* dbg_par) {
    using K = RpKey<I>;
    using T = typename K::T;
    constexpr uint32_t kT = RpHeap<I>::kT;
    const int lane = (int)threadIdx.x;
    const size_t V = (size_t)g.V;
    const size_t slot = blockIdx.x;
    uint4* vr = ws.vrec + slot * V;
    unsigned long long nl[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#if SHD_RP_TIME
    unsigned long long tph[4] = {0, 0, 0, 0}, tlast = wall_clock64();
#endif
    // node storage: ws.nodeCap nodes per slot (replay_layout)
    RpHeap<I> H{reinterpret_cast<typename K::Node*>(ws.node) + slot * (size_t)ws.nodeCap, vr, nl,
                ws.stdPos, ws.stdBase};
    uint32_t* pbuf = ws.pathbuf + slot * (size_t)kMaxHops * 64;
    unsigned long long n_pop = 0, n_push = 0, n_mod = 0, n_rows = 0, n_skip = 0;

    for (;;) {
        uint32_t item = 0;
        if (lane == 0) item = (uint32_t)atomicAdd(&stats[ST_RP_DEQUEUE], 1ull);
        item = rl_u32(item, 0);
        if (item >= (uint32_t)nrows) break;
        const uint32_t row = rows[item];
        const uint32_t src = uni_u32(sources[row]);
        n_rows++;

        // ---- igraph_get_shortest_paths_dijkstra ----
        for (size_t i = (size_t)lane; i < V; i += 64)
            *reinterpret_cast<unsigned long long*>(vr + i) = K::kUnreached;  // dist = -1
        uint32_t size = 1;
        if (lane == 0) {
            K::set_dist(vr + src, T(0));
            H.put(0, K::src_key(), src, RPL_SINK_ST);
        }
        int64_t to_reach = full ? (int64_t)V + 1 : (int64_t)g.ntargets;
        // The root after a sink is the next pop's u unless a shift-up of the relaxation reaches
        // the root: its row bounds (lanes 0, 1) and target word (lane 0) are loaded by vector
        // loads right after the sink and used if it still is (C4-int: every pop).
        uint32_t pf_u = 0xFFFFFFFFu, pf_r = 0, pf_t = 0;
        double dh0 = INFINITY;  // d(landmark) once it is popped (no skip before)
        while (size > 0 && to_reach > 0) {
            // igraph_2wheap_delete_max
            RP_TICK(3);
            const uint32_t u = uni_u32(lds_v<I>(0));
            const T du = K::dist_of_key(K::uni(lds_k<I>(0)));  // mindist = -data[0]
            const double duf = K::f64(du);
            const uint32_t lastp = size - 1u;
            // one round trip: the last node (lane 63) and, independent of the heap, u's target
            // bit, row bounds and first 64 records
            T k1 = K::lo();
            uint32_t v1 = 0;
            if (lane == 63) H.node(lastp, k1, v1, RPL_SINK_LD);
            uint32_t tb, rb, re;
            if (u == pf_u) {
#if SHD_RP_TIME
                nl[13]++;
#endif
                rb = rl_u32(pf_r, 0);
                re = rl_u32(pf_r, 1);
                tb = rl_u32(pf_t, 0);
            } else {
                tb = g.tbits[u >> 5];
                rb = uni_u32(g.rowptr[u]);
                re = uni_u32(g.rowptr[u + 1]);
            }
            uint4 r0 = make_uint4(0u, 0u, 0u, 0u);
            if (rb + (uint32_t)lane < re) r0 = g.rec[rb + (uint32_t)lane];
            size = lastp;
#if SHD_RP_TIME
            nl[7] += size;  // heap size at the pop
#endif
            if (u == (uint32_t)g.landmark) dh0 = duf;
            if (size > 0) rp_pop_sink<I>(H, size, lane, k1, v1);
            n_pop++;
            RP_TICK(0);
            if (size > 0) {
                pf_u = uni_u32(lds_v<I>(0));
                if (lane < 2) pf_r = g.rowptr[pf_u + (uint32_t)lane];
                if (lane == 0) pf_t = g.tbits[pf_u >> 5];
            }
            if ((tb >> (u & 31u)) & 1u) {
                to_reach--;
                // every target is popped: its parent chain is final (relaxing u's edges, as
                // igraph still does, cannot change a popped vertex)
                if (to_reach == 0) break;
            }
            for (uint32_t base = rb; base < re; base += 64) {
                const uint32_t j = base + (uint32_t)lane;
                const bool act = j < re;
                uint32_t t = 0, mypos = 0;
                double w = 0.0;
                T cur = T(0);
                rp_lines(nl, RPL_RELAX_LD, act, g.rec + j);
#if SHD_RP_LINES
                rp_lines(nl, RPL_RELAX_LD, act && !(__dmul_rn(__dadd_rn(dh0, (double)__uint_as_float(g.rec[act ? j : 0].y)), 1.000001) < duf),
                         vr + 4 * (size_t)lane + (act ? g.rec[j].x : 0));
#endif
                bool live = act;
                if (act) {
                    const uint4 r = base == rb ? r0 : g.rec[j];
                    t = r.x;
                    w = __hiloint2double((int)r.w, (int)r.z);
                    // landmark skip: d(t) <= d(h0) + pi(t) (the walk s -> h0 -> t; pi rounded
                    // up, rounding of the sums far inside the 1e-6 margin) below du proves t
                    // popped, and relaxing a popped vertex changes nothing: its record is not read
                    live = !(__dmul_rn(__dadd_rn(dh0, (double)__uint_as_float(r.y)), 1.000001) < duf);
                }
                if (live) {
                    const uint4 x = vr[t];  // {dist, parent slot, heap position}
                    cur = K::dist(x);
                    mypos = x.w;
                }
                n_skip += (unsigned long long)__popcll(__ballot(act && !live));
                const T alt = K::add(du, w);
                const bool first = live && !K::reached(cur);
                const bool impr = live && !first && alt < cur;
                rp_lines(nl, RPL_RELAX_ST, first || impr, vr + 4 * (size_t)lane + t);
                if (first || impr)  // dist and parent in one 12-B store
                    *reinterpret_cast<uint3*>(vr + t) = K::rec(alt, j);
                unsigned long long m = __ballot(first || impr);
                const unsigned long long fm = __ballot(first);
                RP_TICK(1);
                // The step's heap operations run in lane order, but the parent of each one's
                // position is read for all of them in one round trip: a push lands at size + the
                // pushes before it, a modify at its vertex's position.  A read stays valid until
                // an earlier operation moves nodes (dirty) or places its element at that parent.
                uint32_t ppos = 0;
                T pk = K::hi();
                if (first) ppos = size + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
                else if (impr) ppos = mypos;
                // a vertex in the LDS levels: its record's position is only a marker (found by
                // rp_lds_find at its operation, its parent read then)
                bool stale = impr && mypos < kT;
                if ((first || impr) && ppos > 0 && !stale) {
                    uint32_t pv;
                    H.node((ppos - 1u) >> 1, pk, pv, RPL_SHIFT_LD);
                }
                bool dirty = false;
                while (m) {
                    const int l = __ffsll((long long)m) - 1;
                    m &= m - 1ull;
                    const uint32_t tv = rl_u32(t, l);
                    const T xkey = K::key_of(K::rl(alt, l));
                    uint32_t pos;
                    if ((fm >> l) & 1ull) {  // igraph_2wheap_push_with_index
                        if (size >= (uint32_t)V) {  // cannot happen (each vertex queued once)
                            if (lane == 0) atomicAdd(&stats[ST_OVERFLOW], 1ull);
                            dirty = true;
                            continue;
                        }
                        pos = size++;
                        n_push++;
                    } else {  // igraph_2wheap_modify (its sink is a no-op for a larger key)
                        pos = rl_u32(mypos, l);
                        if (pos < kT) pos = rp_lds_find<I>(tv, size, lane);
                        n_mod++;
                    }
                    const bool fresh = (fm >> l) & 1ull;
                    uint32_t mv = 0, mp = 0;
                    int f;
                    if (!dirty && pos > 0 && !__shfl(stale, l)) {
                        if (xkey < K::rl(pk, l)) {  // stays: data[x] < data[parent]
                            if (lane == 0) H.put(pos, xkey, tv, RPL_SHIFT_ST, fresh);
                            f = 0;
                        } else {
                            f = rp_shift_up<I>(H, pos, xkey, tv, lane, mv, mp, fresh, false);
                        }
                    } else {
                        f = rp_shift_up<I>(H, pos, xkey, tv, lane, mv, mp, fresh);
                    }
                    if (f > 0) dirty = true;
                    else if (ppos > 0 && ((ppos - 1u) >> 1) == pos) stale = true;
                    RP_TICK(2);
                    // later lanes whose vertex was moved down by this shift-up
                    for (int i = 0; i < f; ++i) {
                        const uint32_t vi = rl_u32(mv, i), pi = rl_u32(mp, i);
                        if (t == vi) mypos = pi;
                    }
                }
            }
        }

        if (dbg_dist) {  // test hook: the replay's dist / parent vertex in relabelled ids
            for (size_t i = (size_t)lane; i < V; i += 64) {
                const uint4 x = vr[i];
                const T dt = K::dist(x);
                const double d = K::reached(dt) ? K::f64(dt) : -1.0;
                dbg_dist[i] = d;
                dbg_par[i] = (d >= 0.0 && i != src) ? (int32_t)g.own[x.z] : -1;
            }
        }

        // ---- per-target helper (shd-topology.c:561-671) ----
        double rmin = INFINITY;
        const size_t rowbase = (size_t)row * (size_t)A;
        for (int k = lane; k < A; k += 64) {
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
                bool bad = !K::reached(K::dist(vr[t]));
                uint32_t v = t;
                while (!bad && v != src) {
                    const uint32_t j = vr_par(vr, v);
                    if ((int64_t)j >= g.nadj) {
                        bad = true;
                        break;
                    }
                    if (h < (uint32_t)kMaxHops) pbuf[(size_t)h * 64 + lane] = j;
                    h++;
                    v = g.own[j];
                    if (h > (uint32_t)V) bad = true;
                }
                lat = 0.0;
                rel = 1.0;
                rel *= (1.0 - g.vloss[src]);
                rel *= (1.0 - g.vloss[t]);
                if (bad) {
                    atomicAdd(&stats[ST_ERRORS], 1ull);
                    lat = -1.0;
                    rel = -1.0;
                } else {
                    if (h > (uint32_t)kMaxHops) atomicAdd(&stats[ST_LONGPATH], 1ull);
                    for (int x = (int)h - 1; x >= 0; --x) {  // hop x from the target, forwards
                        uint32_t j;
                        if (x < kMaxHops) {
                            j = pbuf[(size_t)x * 64 + lane];
                        } else {
                            uint32_t y = t;  // the chain was validated by the walk above
                            for (int z = 0; z < x; ++z) y = g.own[vr_par(vr, y)];
                            j = vr_par(vr, y);
                        }
                        const double2 hp = g.hop[j];
                        lat = __dadd_rn(lat, hp.x);
                        rel *= (1.0 - hp.y);
                    }
                    if (lat == 0.0) lat = 1.0;
                }
            }
            out_lr[rowbase + (size_t)k] = make_double2(lat, rel);
            out_hops[rowbase + (size_t)k] = (uint16_t)(h > 65535u ? 65535u : h);
            if (lat >= 0.0) rmin = fmin(rmin, lat);
        }
        const unsigned long long mb = wave_min_u64(d2bits(rmin));
        if (lane == 0) {
            if (out_rowmin) out_rowmin[row] = bits2d(mb);
            atomicMin(&stats[ST_GLOBAL_MIN], mb);  // shd-topology.c:500-511
        }
    }
    if (lane == 0) {
        atomicAdd(&stats[ST_RP_POPS], n_pop);
        atomicAdd(&stats[ST_RP_PUSH], n_push);
        atomicAdd(&stats[ST_RP_MOD], n_mod);
        atomicAdd(&stats[ST_RP_ROWS], n_rows);
        atomicAdd(&stats[ST_RP_SKIP], n_skip);
#if SHD_RP_LINES
        for (int i = 0; i < 6; ++i) atomicAdd(&stats[ST_RP_L0 + i], nl[i]);
#endif
#if SHD_RP_TIME
        RP_TICK(3);
        for (int i = 0; i < 4; ++i) atomicAdd(&stats[ST_RP_T0 + i], tph[i]);
        atomicAdd(&stats[ST_RP_T0 + 4], nl[6]);
        atomicAdd(&stats[ST_RP_T0 + 5], nl[7]);
        for (int i = 0; i < 3; ++i) atomicAdd(&stats[ST_RP_T0 + 6 + i], nl[8 + i]);
        atomicAdd(&stats[ST_RP_T0 + 9], nl[13]);
#endif
    }
}

}  // namespace

ReplayLayout replay_layout(int int_keys, uint32_t V) {
    const uint32_t L0 = (uint32_t)replay_lds_levels(int_keys);
    ReplayLayout r;
    r.stdPos = (uint32_t)((1ull << L0) - 1ull);  // positions < kT live in LDS only
    r.stdBase = 0;
    const unsigned long long cap = (unsigned long long)r.stdBase + (V > r.stdPos ? V - r.stdPos : 0u);
    r.nodeCap = (uint32_t)((std::max<unsigned long long>(cap, 64) + 63ull) & ~63ull);  // blocks stay aligned per slot
    return r;
}

int replay_lds_levels(int int_keys) { return int_keys ? SHD_RP_LDS_LEVELS_INT : SHD_RP_LDS_LEVELS; }
int replay_lds_bytes(int int_keys) { return int_keys ? (int)kRpTI * 8 : (int)kRpTF * 12; }

hipError_t launch_heap_replay(const ReplayCSR& g, const ReplayWs& ws, const uint32_t* d_sources,
                              const uint32_t* d_rows, int nrows, const uint32_t* d_targets, int A,
                              int full, double2* out_lr, uint16_t* out_hops, double* out_rowmin,
                              unsigned long long* d_stats, double* dbg_dist, int32_t* dbg_par,
                              hipStream_t stream) {
    const int grid = ws.slots < nrows ? ws.slots : nrows;
    if (grid < 1) return hipSuccess;
    if (g.V <= 0 || (dbg_dist && nrows != 1)) return hipErrorInvalidValue;
    if (g.intKeys)
        hipLaunchKernelGGL(heap_replay_kernel<true>, dim3(grid), dim3(64), 0, stream, g, ws,
                           d_sources, d_rows, nrows, d_targets, A, full, out_lr, out_hops,
                           out_rowmin, d_stats, dbg_dist, dbg_par);
    else
        hipLaunchKernelGGL(heap_replay_kernel<false>, dim3(grid), dim3(64), 0, stream, g, ws,
                           d_sources, d_rows, nrows, d_targets, A, full, out_lr, out_hops,
                           out_rowmin, d_stats, dbg_dist, dbg_par);
    return hipGetLastError();
}

hipError_t preload_replay_module() {
    hipFuncAttributes a;
    const hipError_t e = hipFuncGetAttributes(&a, (const void*)heap_replay_kernel<false>);
    if (e != hipSuccess) return e;
    return hipFuncGetAttributes(&a, (const void*)heap_replay_kernel<true>);
}

}  // namespace shdtopo
