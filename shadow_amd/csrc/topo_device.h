// topo_device.h -- device data layout and kernel launchers (implemented in topo_kernels.hip).
//
// HBM layout (all arrays in the degree-relabelled vertex order, see DESIGN.md "Data layout"):
//   CSR of the undirected topology without self loops:
//     rowptr u32[V+1], adj {u32 col, f64 latency}[2E'] (12-B AoS), aloss f64[2E'] (edge loss)
//   per vertex: vloss f64[V], selfLat f64[V] (NaN = no self loop), selfLoss f64[V]
//   per SSSP slot (one workgroup = one source at a time): 264 B x V of workspace
//   routing table: {f64 lat, f64 rel}[A][A] (16-B records, one gather per packet) + u16 hops
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace shdtopo {

#ifndef SHD_SSSP_BLOCK
#define SHD_SSSP_BLOCK 1024
#endif
constexpr int kSsspBlock = SHD_SSSP_BLOCK;  // threads per SSSP workgroup
#ifndef SHD_BATCH_WGPCU
#define SHD_BATCH_WGPCU 1
#endif
constexpr int kBatchWgPerCu = SHD_BATCH_WGPCU;  // batch-kernel workgroups per CU (share its LDS)
constexpr int kMaxHops = 48;      // per-thread path buffer depth (longer paths: O(h^2) walk)
#ifndef SHD_RING_PER_VERTEX
#define SHD_RING_PER_VERTEX 16
#endif
constexpr int kRingPerVertex = SHD_RING_PER_VERTEX;  // bucket-window entries per slot, in entries
                                                     // per vertex (split evenly over the buckets)
constexpr int kOverPerVertex = 2;  // overflow-pile capacity per slot, in 16-B entries per vertex
                                   // (double buffered: a refill streams the kept entries over)
constexpr int kNearPerVertex = 2; // near-queue capacity per slot, in entries per vertex
#ifndef SHD_KAP_IN_REC
#define SHD_KAP_IN_REC 1
#endif
// 1: the adjacency record's 32-bit field holds {f16 pi(col) rounded up, f16 kappa0(col) rounded
// down} (high, low half), so the batch relaxation gets the target's kappa0 with the record
// instead of a random 4-B load per surviving edge; 0: f32 pi(col) rounded up, kappa0 from g.kap0
constexpr bool kKapInRec = SHD_KAP_IN_REC != 0;
#ifndef SHD_KPROBES
#define SHD_KPROBES 8
#endif
// kappa probes per vertex (4 or 8): the batch kernel's cut of a kappa-sorted row needs a
// binary search (dependent loads) only past the last probe
constexpr int kKProbes = SHD_KPROBES;
static_assert(kKProbes == 4 || kKProbes == 8, "kappa probes");

// indices into the device stats block (unsigned long long[16])
enum StatIdx {
    ST_GLOBAL_MIN = 0,  // f64 bits of the min latency over every computed pair
    ST_AMBIGUOUS = 1,   // pairs whose parent chain crosses a d-tied parent
    ST_RELAX = 2,       // edge relaxations attempted
    ST_LONGPATH = 3,    // pairs longer than kMaxHops
    ST_ERRORS = 4,      // pairs with a missing edge / unreachable target
    ST_DEQUEUE = 5,     // next source to take (persistent workgroups)
    ST_OVERFLOW = 6,    // queue overflow / iteration guard tripped
    ST_T_INIT = 7,      // wall-clock ticks summed over workgroups: distance init
    ST_T_SSSP = 8,      //   near-far SSSP
    ST_T_PARENT = 9,    //   parent derivation for the target chains
    ST_T_TARGET = 10,   //   per-target latency / reliability / hops
    ST_NEAR_IT = 11,    // near-phase iterations
    ST_SPLITS = 12,     // buckets taken from the bucket window
    ST_EV0 = 13,        // event counters (ShdStats.events): queue entries expanded, tail
                        // relaxations, tail improvements, window entries taken, overflow entries
                        // refilled, parent-pass vertices, relaxations onto settled tail vertices,
                        // stale entries skipped
    ST_FARSCAN = 21,    // sources that overflowed a queue (finished with scanning buckets)
    ST_T_SPLIT = 22,    // wall-clock ticks summed over workgroups: bucket changes + refills
    ST_OVERSITE = 23,   // OR of the push sites that overflowed (diagnostic)
    ST_RP_DEQUEUE = 24, // heap replay: next row to take (persistent wavefronts)
    ST_RP_POPS = 25,    //   heap pops (delete_max) summed over replayed rows
    ST_RP_PUSH = 26,    //   pushes (first reach)
    ST_RP_MOD = 27,     //   modifies (strict improvement of a queued vertex)
    ST_RP_ROWS = 28,    //   rows replayed
    ST_ROUTE_BAD = 29,  // packets with a column outside [0, A) (not routed) since the last build
    ST_PT0 = 30,        // batch kernel parent pass, wall ticks summed over workgroups: walks,
                        //   merged row scans, recount + finalize, next level (4 slots)
    ST_RP_L0 = 34,      // replay 64-B lines (SHD_RP_LINES builds): sink ld/st, shift-up ld/st,
                        // relaxation ld/st
    ST_RP_T0 = 40,      // replay wall ticks (SHD_RP_TIME builds): sink, loads, heap ops, rest
                        // + sink rounds, heap size summed over pops, sink sub-phases
                        // (LDS walk, HBM rounds, moves), root-prefetch hits
    ST_RP_SKIP = 50,    // replay relaxations whose vertex record the landmark skip did not read
    ST_BT0 = 51,        // batch kernel (SHD_BATCH_TIME builds): wave ticks of tail iterations in
                        // chunk loads / phase A / phase B, the same for hub iterations, phase-B
                        // rounds, surviving edges (8 slots)
    ST_COUNT = 59
};

struct DevCSR {
    int32_t V = 0;
    int64_t nadj = 0;
    const uint32_t* rowptr = nullptr;
    const uint32_t* adj = nullptr;  // 16-B AdjRec {u32 col, f32 pi(col) rounded up, f64 wt}
    const uint32_t* adjk = nullptr; // the same records, each row sorted by kappa = w - pi(col)
    const float* kap = nullptr;     // kappa of adjk (f32 rounded down; -inf: pi unknown)
    const float4* ksum = nullptr;   // per vertex: kappa at row positions 0, 1, 3, 7[, 15, 31, 63,
                                    // 127] (kKProbes floats, +inf past the row)
    const float* kap0 = nullptr;    // per vertex: smallest kappa of its row (+inf: empty row)
    const uint32_t* spt = nullptr;  // per vertex {h0-tree parent, its slot of (parent, v), f64 w}
    double piMax = 0.0;             // largest finite pi
    const double* aloss = nullptr;
    const double* vloss = nullptr;
    const double* selfLat = nullptr;
    const double* selfLoss = nullptr;
    int rows_sorted = 0;  // adjacency rows ascending by neighbour (enables binary row search)
    // bit 30 of adjk's column word marks an attached vertex (a table target); the batch
    // relaxation then skips pairs into non-target tail vertices that would expand nothing
    int tflags = 0;
};

// per-slot workspace, slot-major: array + slot * V
struct SlotWs {
    int slots = 0;
    int64_t V = 0;
    unsigned long long* dist = nullptr;  // f64 bits, +inf = unreached
    uint32_t* stamp = nullptr;           // near-queue / chain-queue dedupe (iteration id)
    unsigned long long* qa = nullptr;  // near queues: (hi32 of the pushed distance << 32) |
    unsigned long long* qb = nullptr;  // vertex, kNearPerVertex * V entries (no dedupe)
    unsigned long long* ring = nullptr;  // bucket window: kRingPerVertex * V entries, same format
    unsigned long long* over = nullptr;  // overflow pile (buckets past the window), 2 buffers of
                                         // kOverPerVertex * V {u64 key, u64 vertex} entries
    unsigned long long* best = nullptr;  // parent pass: min d[u] over candidates
    uint32_t* cnt = nullptr;             // parent pass: candidates at the min
    uint32_t* bslot = nullptr;           // parent pass: lowest adjacency slot at the min
    unsigned long long* memo = nullptr;  // (source epoch << 32) | ambiguous << 31 | slot
    uint32_t* par = nullptr;             // parent vertex
    uint32_t* pathbuf = nullptr;         // [slot][kMaxHops][kSsspBlock]
    uint32_t* counters = nullptr;        // [slot][4]: iteration id, (unused), source epoch
    // batched kernel (sssp_batch_kernel, K sources per slot): dist is [V][K] per slot, ring holds
    // ring_entries u32 entries per slot (the parent pass' pair list; no overflow pile:
    // over_entries is 0); qa / qb hold q_stride u64 per slot (near queues, parent pair lists of
    // V * K u32); stamp/best/cnt/bslot/memo/par are per (vertex, source) pair, V * K per slot;
    // mask = 2 parities of a K-bit mask per vertex; hpar [P][K] parent hints
    int K = 1;
    int64_t q_stride = 0;
    int64_t ring_entries = 0;
    int64_t over_entries = 0;
    uint8_t* mask = nullptr;
    uint32_t* hpar = nullptr;
    // per row of the launch: set to 1 when a pair of the row crosses a d-tied parent (its parent
    // chain needs igraph's heap pop order: the row is recomputed by heap_replay_kernel)
    uint8_t* rowflag = nullptr;
    // batch kernel: output row of batch position p (sources are taken in a locality order, the
    // table keeps row order); nullptr = identity
    const uint32_t* rowmap = nullptr;
    // diagnostic (SHD_BATCH_TRACE): per batch {wall_clock64 at dequeue, at its end, slot}
    unsigned long long* btrace = nullptr;
};

// Incidence-order CSR of the heap replay (topo_replay.hip), relabelled vertex ids: row x holds
// x's neighbours in igraph_incident order (ascending ORIGINAL neighbour id; directed graphs:
// out-neighbours), self loops dropped, parallel edges merged.
//   rec  {u32 col, u32 row vertex x, f64 latency (min over a parallel group)}   16 B
//   hop  {f64 latency, f64 packet loss} of the igraph_get_eid edge (lowest edge id)  16 B
struct ReplayCSR {
    int32_t V = 0;
    int64_t nadj = 0;
    const uint32_t* rowptr = nullptr;
    // {u32 neighbour, f32 pi(neighbour) rounded up (+inf: no landmark), f64 w} per entry
    const uint4* rec = nullptr;
    const uint32_t* own = nullptr;  // row (vertex) of each entry: the epilogue's parent walk
    const double2* hop = nullptr;
    const double* vloss = nullptr;
    const double* selfLat = nullptr;
    const double* selfLoss = nullptr;
    const uint32_t* tbits = nullptr;  // target (attached vertex) bitmap over V
    int64_t ntargets = 0;             // distinct targets (igraph's to_reach)
    int32_t landmark = -1;            // vertex the rec pi values are measured from (-1: none)
};

// per-slot workspace of the heap replay (one wavefront = one slot), slot-major [slot][V]:
// vertex records {f64 dist (-1 = unreached), u32 parent (replay-CSR slot of the parent edge),
// u32 heap position} and heap nodes {f64 key, u32 vertex, pad} (positions >= the LDS part),
// 16 B each (one line per access), and a path buffer [kMaxHops][64] per slot.
// 32 B x V + 12 KiB per slot.
struct ReplayWs {
    int slots = 0;
    uint4* vrec = nullptr;
    uint4* node = nullptr;
    uint32_t* pathbuf = nullptr;
};

// LDS plan of one SSSP workgroup: H hub distance words (+ their queue bitmaps) and P parent
// hints, sized to the workgroup's share of the CU's 160 KiB (wg_per_cu workgroups per CU).
struct SsspLdsPlan {
    uint32_t H = 0;     // LDS-resident hub distances (vertex ids 0..H-1 after the relabel)
    uint32_t P = 0;     // hubs with parent hints (P <= H)
    size_t bytes = 0;   // dynamic LDS per workgroup
};
// hub_limit: cap on H (-1 = as many as fit); V: vertices of the graph (H <= V)
SsspLdsPlan sssp_lds_plan(int wg_per_cu, int64_t hub_limit, uint32_t par_hubs, int64_t V);

hipError_t launch_sssp_rows(const DevCSR& g, const SlotWs& ws, const uint32_t* d_sources,
                            int nsrc, const uint32_t* d_targets, int A, double delta,
                            const SsspLdsPlan& plan, uint32_t far_cap,
                            uint32_t near_cap, bool events,
                            double2* out_lr,
                            uint16_t* out_hops, double* out_rowmin, unsigned long long* d_stats,
                            hipStream_t stream);

// Batched multi-source SSSP (topo_sssp_batch.hip): K in {2, 4, 8, 16} sources per workgroup in
// lock-step over buckets of d + srcsh[row] (srcsh >= 2 delta).  plan from sssp_batch_lds_plan.
// kf (1..K): sources per batch (batch b = positions [b kf, b kf + kf)).
SsspLdsPlan sssp_batch_lds_plan(int K, int64_t hub_limit, uint32_t par_hubs, int64_t V);
// bit 30 of every adjk column word := the column is set in tbits (the attached vertices)
hipError_t launch_mark_targets(uint32_t* adjk, int64_t nadj, const uint32_t* tbits,
                               hipStream_t stream);
// target-aware kappa fixpoint (topo_sssp_batch.hip): one step K_out = F(K_in) (K_in nullptr:
// kappa0), then the f16 kappa field of the relaxation copy's records := K(column)
hipError_t launch_kfix_step(const uint32_t* rowptr, const uint32_t* adj, const double* pot,
                            const uint32_t* tbits, const double* Kin, double* Kout, int64_t V,
                            unsigned int* changed, hipStream_t stream);
hipError_t launch_kfix_store(uint32_t* adjk, int64_t nadj, const double* K, hipStream_t stream);
// re-sort every row of the relaxation copy (records, kappa array, probes, kappa0) by the
// target-aware key kap' of the current target set (tbits) and K
hipError_t launch_kprime_resort(uint32_t* adjk, float* kap, float* ksum, float* kap0,
                                const uint32_t* rowptr, int64_t V, int64_t nadj, const double* pot,
                                const uint32_t* tbits, const double* K, hipStream_t stream);
hipError_t launch_sssp_batch(int K, const DevCSR& g, const SlotWs& ws, const uint32_t* d_sources,
                             const double* d_srcsh, int nsrc, int kf, const uint32_t* d_targets, int A,
                             double delta, const SsspLdsPlan& plan, uint32_t far_cap,
                             double2* out_lr, uint16_t* out_hops, double* out_rowmin,
                             unsigned long long* d_stats, hipStream_t stream);

// Exact igraph-0.7 Dijkstra replay, one wavefront per row (topo_replay.hip): rows[0..nrows) index
// d_sources / the output rows.  full = 1 ignores the early exit (test hook); dbg_dist / dbg_par
// (V entries, nrows == 1) receive the replay's distances and parent vertices (relabelled ids).
hipError_t launch_heap_replay(const ReplayCSR& g, const ReplayWs& ws, const uint32_t* d_sources,
                              const uint32_t* d_rows, int nrows, const uint32_t* d_targets, int A,
                              int full, double2* out_lr, uint16_t* out_hops, double* out_rowmin,
                              unsigned long long* d_stats, double* dbg_dist, int32_t* dbg_par,
                              hipStream_t stream);
int replay_lds_levels();
int replay_lds_bytes();  // LDS of one replay wavefront (its heap's top levels)

hipError_t launch_pair_table_complete(int A, int64_t row0, int64_t rows, const double* elatAA,
                                      const double* elossAA, const double* vlossA, double2* out_lr,
                                      uint16_t* out_hops, double* out_rowmin,
                                      unsigned long long* d_stats, hipStream_t stream);

hipError_t launch_packet_route(int64_t n, const int32_t* src, const int32_t* dst,
                               const uint32_t* payload, const uint32_t* state_in,
                               const uint64_t* now, const double2* table, int64_t A,
                               uint64_t jump, int clamp, uint64_t* t_out, uint32_t* state_out,
                               uint8_t* delivered, unsigned long long* d_bad, hipStream_t stream);

hipError_t launch_row_min(int64_t rows, int64_t A, const double2* lr, double* out_rowmin,
                          hipStream_t stream);

hipError_t launch_fill_u64(unsigned long long* p, unsigned long long v, int64_t n,
                           hipStream_t stream);

// SSSP workgroups one CU holds with the LDS plan of wg_per_cu (registers and LDS permitting)
int sssp_max_blocks_per_cu(int wg_per_cu);

}  // namespace shdtopo
