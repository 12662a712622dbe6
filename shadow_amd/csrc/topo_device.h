// topo_device.h -- device data layout and kernel launchers (implemented in topo_kernels.hip).
//
// HBM layout (all arrays in the degree-relabelled vertex order, see DESIGN.md "Data layout"):
//   CSR of the undirected topology without self loops:
//     rowptr u32[V+1], adj {u32 col, u32 pi / kappa0 field, f64 latency}[2E'] (16-B AoS), its
//     kappa-sorted copy adjk, aloss f64[2E'] (edge loss)
//   per vertex: vloss f64[V], selfLat f64[V] (NaN = no self loop), selfLoss f64[V], pi f64[V]
//   per SSSP slot (one workgroup = K sources at a time): DESIGN.md 3.2
//   routing table: {f64 lat, f64 rel}[A][A] (16-B records, one gather per packet) + u16 hops
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

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
// doubles of the batch kernel's path buffer per slot: the chain losses [kMaxHops][kSsspBlock]
constexpr size_t kPathBufPerSlot = (size_t)kMaxHops * kSsspBlock;
// parent pass: pairs of one row-scan chunk by default (records per slot: chunk x K, one per
// merged vertex and source; C4 sends ~2.6 k pairs per level of a batch to row scans)
constexpr uint32_t kRowScanCap = 16384;
// the candidate count of a row-scan record no pair asked for
constexpr uint32_t kRsUnreq = 0xFFFFFFFEu;
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
    ST_TOUCHED = 59,    // tail distance lines reset at batch starts (lines the batches touched)
    ST_WALK = 60,       // batch kernel parent pass: walk steps (pairs claimed and resolved)
    ST_WK0 = 61,        //   of which resolved by the h0-tree guess, by a tail's improver, by a
                        //   hub's improver, and pairs sent to row scans (4 slots)
    ST_SW0 = 65,        // batch kernel sweeps (SHD_BATCH_TIME builds): pending tail vertices
                        //   visited, of which queued (a pair in the opened bucket), holding a
                        //   pair in that bucket that the kappa test kept out, kept pending
    ST_WL0 = 69,        // batch kernel (SHD_BATCH_WRCOUNT builds): 64-B lines written per
                        //   category (16 slots, topo_sssp_batch.hip WL_*)
    ST_RL0 = 85,        //   then 64-B lines read per category (8 slots, RL_*)
    ST_COUNT = 93
};

// A directed topology (igraph mode OUT, shd-topology.c:762-763) relaxes out-edges but finds a
// vertex's parent among its in-edges: rowptr / adjk / kap / ksum / kap0 are the OUT rows,
// rowptr_in / adj / aloss the IN rows (the parent pass).  Undirected: rowptr_in == rowptr.
struct DevCSR {
    int32_t V = 0;
    int64_t nadj = 0;
    const uint32_t* rowptr = nullptr;     // rows of adjk (relaxation)
    const uint32_t* adj = nullptr;  // 16-B AdjRec {u32 col, f32 pi(col) rounded up, f64 wt}
    const uint32_t* adjk = nullptr; // the relaxation records, each row sorted by kappa = w - pi(col)
    const float* kap = nullptr;     // kappa of adjk (f32 rounded down; -inf: pi unknown)
    const float4* ksum = nullptr;   // per vertex: kappa at row positions 0, 1, 3, 7[, 15, 31, 63,
                                    // 127] (kKProbes floats, +inf past the row)
    const float* kap0 = nullptr;    // per vertex: smallest kappa of its row (+inf: empty row)
    // per vertex, 32 B: {h0-tree parent, its slot in v's row, f64 w, f64 packet loss of that
    // edge, pad} (one line per walk hop)
    const uint32_t* spt = nullptr;
    double piMax = 0.0;             // largest finite pi
    const double* aloss = nullptr;
    const double* vloss = nullptr;
    const double* selfLat = nullptr;
    const double* selfLoss = nullptr;
    int rows_sorted = 0;  // adjacency rows ascending by neighbour (enables binary row search)
    // bit 30 of adjk's column word marks an attached vertex (a table target); the batch
    // relaxation then skips pairs into non-target tail vertices that would expand nothing
    int tflags = 0;
    // (last: the undirected kernel's argument layout stays that of the fields above)
    int directed = 0;
    const uint32_t* rowptr_in = nullptr;  // rows of adj / aloss (parent pass)
};

// per-slot workspace of the batched SSSP (sssp_batch_kernel, K sources per slot), slot-major:
// array + slot * V [* K]
struct SlotWs {
    int slots = 0;
    int64_t V = 0;
    unsigned long long* dist = nullptr;  // [V][K] f64 bits, +inf = unreached (rows < H unused)
    uint4* prec = nullptr;               // [V][K] pair records {parent | amb << 31 | bad << 30,
                                         // batch tag, f64 loss of the parent edge}
    unsigned long long* qa = nullptr;    // near queues / parent pair lists (q_stride u64 per slot)
    unsigned long long* qb = nullptr;
    uint32_t* ring = nullptr;            // ring_entries u32 per slot: parent pair list, vertex
                                         // list, pending bitmap, tie bitmap
    uint4* rscan = nullptr;              // parent pass, rs_chunk x K per slot: per (merged vertex,
                                         // source) of a row-scan chunk {min d[u] over the candidates
                                         // (u64), candidates at the min, lowest adjacency slot}
    uint32_t rs_chunk = kRowScanCap;     // pairs per row-scan chunk (option "row_scan_chunk")
    double* pathbuf = nullptr;           // [slot][kPathBufPerSlot]: edge losses of a path
    uint32_t* counters = nullptr;        // [slot][4]: batch tag, (unused)
    int K = 8;
    int64_t q_stride = 0;
    int64_t ring_entries = 0;
    uint8_t* mask = nullptr;             // 2 parities of a K-bit source mask per vertex
    uint32_t* hpar = nullptr;            // [P][K] parent hints of the LDS hubs
    // per row of the launch: set to 1 when a pair of the row crosses a d-tied parent (its parent
    // chain needs igraph's heap pop order: the row is recomputed by heap_replay_kernel)
    uint8_t* rowflag = nullptr;
    // output row of batch position p (sources are taken in a locality order, the table keeps
    // row order); nullptr = identity
    const uint32_t* rowmap = nullptr;
    // diagnostic (SHD_BATCH_TRACE): per batch kBTraceWords u64 {wall_clock64 at dequeue, at its
    // end, slot, near iterations, sweeps, expansions, relaxations, sources, ticks at the SSSP's,
    // the parent pass' and the epilogue's end, 0}
    unsigned long long* btrace = nullptr;
    // batch layout (option balance, topo_core.cpp): batch b takes positions [bstart[b],
    // bstart[b + 1]) (at most K), nbat batches; nullptr = batch b takes [b kf, b kf + kf)
    const uint32_t* bstart = nullptr;
    int nbat = 0;
};
constexpr int kBTraceWords = 12;  // u64 words per batch of SlotWs::btrace (per-batch trace / costs)

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
    // 1: u32 heap keys (every latency an integer, V x max latency < 2^32 - 1: exact, see
    // topo_replay.hip RpKey); 0: f64 keys
    int32_t intKeys = 0;
};

// per-slot workspace of the heap replay (one wavefront = one slot), slot-major [slot][V]:
// vertex records {f64 dist (-1 = unreached), u32 parent (replay-CSR slot of the parent edge),
// u32 heap position} and heap nodes {f64 key, u32 vertex, pad} (positions >= the LDS part),
// 16 B each (one line per access; u32 keys: {u32 dist, pad, ...} and 8-B nodes {u32 key, u32
// vertex}, the node block then V x 8 B per slot), and a path buffer [kMaxHops][64] per slot.
// 32 B (u32 keys: 24 B) x V + 12 KiB per slot.
struct ReplayWs {
    int slots = 0;
    uint4* vrec = nullptr;
    uint4* node = nullptr;     // nodeCap heap nodes per slot (node size: 8 B u32 keys, 16 B f64)
    uint32_t* pathbuf = nullptr;
    uint32_t nodeCap = 0;      // physical heap nodes per slot (replay_layout)
    uint32_t stdPos = 0;       // first heap position stored position-major (past the blocked bands)
    uint32_t stdBase = 0;      // its physical node index
};
// Physical layout of a replay heap's HBM levels (topo_replay.hip, RpHeap::phys): the levels below the
// LDS ones in bands of one sink round's height, each band root's subtree contiguous; the levels
// past the last band the heap can fill, position-major.
struct ReplayLayout {
    uint32_t stdPos, stdBase, nodeCap;
};
ReplayLayout replay_layout(int int_keys, uint32_t V);

// Hub rows (ids < rows: the long rows of the degree order) cut into segments of at most kHubSeg
// entries, one wavefront each in the row-parallel steps (graph preparation, the target-aware
// kappa fixpoint): the longest rows (250 k entries on C4) no longer serialise on one wavefront.
// A row cut into several segments leaves one partial result per segment, combined by a
// finalize pass over `multi`.
constexpr uint32_t kHubSeg = 4096;
struct HubSegs {
    uint32_t rows = 0;             // hub rows [0, rows); the rest take a thread each
    const uint2* seg = nullptr;    // {row, first entry} per segment, rows ascending
    uint32_t nseg = 0;
    const uint4* multi = nullptr;  // {row, first segment, segments, 0} of the rows cut in several
    uint32_t nmulti = 0;
};
// the segment tables of rows [0, rows) from the first rows + 1 entries of rowptr (host)
void hub_segments(const uint32_t* rowptr_head, uint32_t rows, std::vector<uint2>& seg,
                  std::vector<uint4>& multi);

// LDS plan of one batched SSSP workgroup: H hub distance rows (+ their queue masks) and P
// parent hints, sized to the CU's 160 KiB.
struct SsspLdsPlan {
    uint32_t H = 0;     // LDS-resident hub distances (vertex ids 0..H-1 after the relabel)
    uint32_t P = 0;     // hubs with parent hints (P <= H)
    size_t bytes = 0;   // dynamic LDS per workgroup
};

// Batched multi-source SSSP (topo_sssp_batch.hip): K in {2, 4, 8, 16} sources per workgroup in
// lock-step over buckets of d + srcsh[row] (srcsh >= 2 delta).  plan from sssp_batch_lds_plan.
// kf (1..K): sources per batch (batch b = positions [b kf, b kf + kf)).
SsspLdsPlan sssp_batch_lds_plan(int K, int64_t hub_limit, uint32_t par_hubs, int64_t V);
// bit 30 of every adjk column word := the column is set in tbits (the attached vertices)
hipError_t launch_mark_targets(uint32_t* adjk, int64_t nadj, const uint32_t* tbits,
                               hipStream_t stream);
// target-aware kappa fixpoint (topo_sssp_batch.hip): kap_e = every out-row entry's w - pi(y)
// (static: once per graph); one step K_out = F(K_in) (K_in nullptr: kappa0), K buffers of 2 V
// doubles [K | Kt = target ? -inf : K]; then the f16 kappa field of the relaxation copy's records
// := K(column).  part: scratch of hs.nseg doubles (the per-segment minima of cut rows)
hipError_t launch_kfix_kap(const uint32_t* adj, const double* pot, int64_t nadj, double* kap,
                           hipStream_t stream);
hipError_t launch_kfix_step(const uint32_t* rowptr, const uint32_t* adj, const double* kap_e,
                            const uint32_t* tbits, const double* Kin, double* Kout, int64_t V,
                            const HubSegs& hs, double* part, unsigned int* changed,
                            hipStream_t stream);
hipError_t launch_kfix_store(uint32_t* adjk, int64_t nadj, const double* K, hipStream_t stream);
// re-sort every row of the relaxation copy (records, kappa array, probes, kappa0) by the
// target-aware key kap' of the current target set (tbits) and K.  Scratch (KprimeScratch, sized
// by kprime_scratch_bytes) is the caller's, so the resort allocates nothing and never syncs.
// rows of at most kSegBlock entries are sorted in LDS; the longer ones' entries, listed once per
// graph row by row (pos: adjacency position, row: the row's ordinal among the long rows), go
// through a device-wide radix sort of (ordinal << 32 | key) -- end_bit = 32 + bits of the ordinal
constexpr uint32_t kSegBlock = 4096;
struct SegBig {
    const uint32_t* pos = nullptr;
    const uint32_t* row = nullptr;
    int64_t nitems = 0;
    int end_bit = 33;
    unsigned long long* keys = nullptr;  // 2 x nitems
    uint32_t* vals = nullptr;            // 2 x nitems
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
};
struct KprimeScratch {
    float* key = nullptr;       // nadj
    uint32_t* idx = nullptr;    // nadj: each sorted entry's source position
    uint4* rec = nullptr;       // nadj
    SegBig big;                 // the rows longer than kSegBlock (listed once per graph)
};
// segmented sort (ascending f32 keys, stable, hipcub's order): rows <= 64 by waves, <= kSegBlock
// by workgroups in LDS, the longer rows' entries by one device-wide radix sort
hipError_t segsort_big_tmp_bytes(int64_t nitems, int end_bit, size_t* bytes);
hipError_t launch_segsort(const uint32_t* rowptr, int64_t V, int64_t nadj, const float* key,
                          float* key_out, uint32_t* idx_out, const SegBig& big, hipStream_t stream);
hipError_t segsort_reference(const uint32_t* rowptr, int64_t V, int64_t nadj, const float* key,
                             const uint32_t* idx_in, float* key_out, uint32_t* idx_out, void* tmp,
                             size_t* tmp_bytes, hipStream_t stream);
hipError_t preload_kprime_sort(hipStream_t stream);
hipError_t launch_kprime_resort(uint32_t* adjk, float* kap, float* ksum, float* kap0,
                                const uint32_t* rowptr, int64_t V, int64_t nadj, const double* pot,
                                const uint32_t* tbits, const double* K, const KprimeScratch& sc,
                                hipStream_t stream);
hipError_t launch_sssp_batch(int K, const DevCSR& g, const SlotWs& ws, const uint32_t* d_sources,
                             const double* d_srcsh, int nsrc, int kf, const uint32_t* d_targets, int A,
                             double delta, const SsspLdsPlan& plan, uint32_t iter_guard,
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
int replay_lds_levels(int int_keys);
int replay_lds_bytes(int int_keys);  // LDS of one replay wavefront (its heap's top levels)

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
// p[b * stride + i] = v for b < nb, i < n
hipError_t launch_fill_u64_strided(unsigned long long* p, unsigned long long v, int64_t nb,
                                   int64_t stride, int64_t n, hipStream_t stream);

// ---- graph preparation on the GPU (topo_prep.hip), once per topology: DESIGN.md 3.1 ----
// Input arrays are the parsed graph in HBM (document order: eu / ev int32[E], elat / eloss f64[E],
// vloss f64[V]); outputs are in the relabelled vertex order.  Each call synchronises `st`.
// degrees of the non-loop graph (deg u32[V], in + out when directed), the lowest-id self loop
// (selfE, ~0 = none) and *nadj = 2 x non-loop edges
hipError_t prep_degrees(int64_t V, int64_t E, const int32_t* eu, const int32_t* ev, uint32_t* deg,
                        uint32_t* selfE, int64_t* nadj, hipStream_t st);
// relabel (degree descending, the tail grouped by its primary hub among the first H): perm
// (new -> old), inv (old -> new), rowptr u32[V+1], per-vertex loss and self-loop arrays
hipError_t prep_relabel(int64_t V, int64_t E, uint32_t H, const int32_t* eu, const int32_t* ev,
                        const uint32_t* deg, const uint32_t* selfE, const double* elat,
                        const double* eloss, const double* vloss_in, uint32_t* perm,
                        uint32_t* inv, uint32_t* rowptr, double* vloss, double* selfLat,
                        double* selfLoss, hipStream_t st);
// 16-B adjacency records {col, 0, f64 w} rows ascending by (neighbour, edge id), and aloss
// (nullable).  mode 0: every non-loop edge in both rows (undirected, nadj = 2E'); 1: out-rows
// only, 2: in-rows only (directed, nadj = E'); for modes 1 and 2 rowptr (u32[V+1]) is counted
// from the entries
enum { kAdjBoth = 0, kAdjOut = 1, kAdjIn = 2 };
hipError_t prep_adjacency(int64_t V, int64_t E, int64_t nadj, const int32_t* eu, const int32_t* ev,
                          const uint32_t* inv, const double* elat, const double* eloss,
                          uint32_t* adj, double* aloss, hipStream_t st, int mode = kAdjBoth,
                          uint32_t* rowptr = nullptr);
// pi = d(h0, .) from vertex 0 (f64[V], +inf = unreached); *iterations = frontier rounds
hipError_t prep_h0_distances(int64_t V, const uint32_t* rowptr, const uint32_t* adj, double* pot,
                             int* iterations, hipStream_t st);
// h0 tree (sptPar u32[V], spt {parent, slot in v's row, f64 w, f64 loss, pad} 32 B [V]), the
// records' pi / kappa0 field, *piMax = the largest finite pi; hub rows by segments (hs).
// what: kTreeParents (the tree, from rows of candidate parents: in-rows when directed) |
// kTreeKappa (kappa0 and the records' field, from relaxation rows: out-rows when directed)
enum { kTreeParents = 1, kTreeKappa = 2 };
hipError_t prep_tree(int64_t V, int64_t nadj, const HubSegs& hs, const uint32_t* rowptr,
                     uint32_t* adj, const double* aloss, const double* pot, uint32_t* sptPar,
                     uint32_t* spt, double* piMax, hipStream_t st,
                     int what = kTreeParents | kTreeKappa);
// the plain kappa-sorted relaxation copy (adjk, kap, ksum, kap0) of adj: also restores it after
// a target-aware re-sort when the target-aware order no longer applies
hipError_t launch_kappa_copy(int64_t V, int64_t nadj, const HubSegs& hs, const uint32_t* rowptr,
                             const uint32_t* adj, const double* pot, const uint32_t* sptPar,
                             uint32_t* adjk, float* kap, float* ksum, float* kap0,
                             hipStream_t st);

// the heap replay's incidence CSR (ReplayCSR) from the parsed edges in HBM: rows in relabelled
// ids, each in igraph_incident order (ascending original neighbour; parallel groups merged, the
// lowest edge id's latency / loss for the hop, the group's minimum latency for the heap).
// rec / own / hop hold up to 2E (E directed) entries; *nrec = the entries written.
hipError_t prep_replay_csr(int64_t V, int64_t E, int directed, const int32_t* eu,
                           const int32_t* ev, const double* elat, const double* eloss,
                           const uint32_t* inv, const double* pot, uint32_t* rowptr, uint4* rec,
                           uint32_t* own, double2* hop, int64_t* nrec, hipStream_t st);

// Load each kernel module's code object now (dev_init) instead of at its first launch inside
// the first build: the runtime loads code objects lazily.
hipError_t preload_batch_module();
hipError_t preload_prep_module();
hipError_t preload_kernels_module();
hipError_t preload_replay_module();

}  // namespace shdtopo
