/*
 * shd_topology_abi.h -- C ABI of libshdtopo.so, the MI355X-native routing engine that replaces
 * Shadow's topology subsystem (src/topology/shd-topology.c + shd-path.c, Shadow v1.11.1).
 *
 * Part 1 is exactly the reference header src/topology/shd-topology.h:12-22 with the GLib
 * typedefs written as plain C (gchar=char, gboolean=int, gdouble=double, guint64=uint64_t), so
 * Shadow's callers link against it unchanged:
 *   runnable/action/shd-load-topology.c:50,79  topology_new
 *   engine/shd-slave.c:147                     topology_free
 *   host/shd-host.c:97 / :172 / :1082          topology_attach / topology_detach / isRoutable
 *   engine/shd-worker.c:352,360                topology_getReliability / topology_getLatency
 *   engine/shd-slave.c:261-268                 topology_getLatency (TCP autotune)
 *
 * Imports resolved from the Shadow executable at load time (weak: a standalone process loads
 * libshdtopo_shim.so, a restatement of these four functions, first):
 *   uint32_t address_toNetworkIP(Address*)       src/topology/shd-address.c:114
 *   double   random_nextDouble(Random*)          src/utility/shd-random.c:34
 *   void     worker_updateMinTimeJump(double)    src/engine/shd-worker.c:459
 *
 * Part 2 adds the two entry points the north star names: the global minimum
 * latency (absent in the reference: it is pushed from shd-topology.c:500-511, K2) and the
 * per-window packet batch (engine-side adapter of src/engine/shd-worker.c:332-370).
 *
 * Part 3 is the device-level boundary used by multi-GPU drivers (one process per GPU): shard
 * rows into caller-owned HBM buffers, install an all-gathered table, route packets already
 * resident in HBM.  Device pointers are plain `void*` / typed pointers into HBM; `stream` is a
 * hipStream_t passed as void* (NULL = the library's own stream).  No torch types anywhere.
 *
 * Errors follow the reference: getters return -1.0 for an unattached address
 * (shd-topology.c:882-892, logs "critical"); an attached-but-unroutable pair is a fatal
 * error() in the reference (shd-topology.c:917-928) -- here it aborts too unless the
 * "abort_on_error" option is set to 0, in which case the getter returns -1.0.
 */
#ifndef SHD_TOPOLOGY_ABI_H_
#define SHD_TOPOLOGY_ABI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct _Topology Topology;
typedef struct _Address Address; /* Shadow's, opaque here */
typedef struct _Random Random;   /* Shadow's, opaque here */

/* ---------------- Part 1: src/topology/shd-topology.h:14-22 ---------------- */
/* shd-topology.c:1237  NULL on failure (parse error, not strongly connected, latency <= 0) */
Topology* topology_new(const char* graphPath);
/* shd-topology.c:1199 */
void topology_free(Topology* top);
/* shd-topology.c:1154  consumes exactly one random_nextDouble(randomSourcePool) unless LPM */
void topology_attach(Topology* top, Address* address, Random* randomSourcePool, char* ipHint,
                     char* geocodeHint, char* typeHint, uint64_t* bwDownOut, uint64_t* bwUpOut);
/* shd-topology.c:1190 */
void topology_detach(Topology* top, Address* address);
/* shd-topology.c:960 */
int topology_isRoutable(Topology* top, Address* srcAddress, Address* dstAddress);
/* shd-topology.c:940  ms, -1.0 on failure */
double topology_getLatency(Topology* top, Address* srcAddress, Address* dstAddress);
/* shd-topology.c:950  [0,1], -1.0 on failure */
double topology_getReliability(Topology* top, Address* srcAddress, Address* dstAddress);

/* ---------------- Part 2: north-star additions ---------------- */
/* Global min latency (ms) over all attached pairs incl. self pairs; replaces the lazily
 * pushed minimum of shd-topology.c:500-511.  Builds the table if needed.  -1.0 on failure. */
double topology_getMinimumLatency(Topology* top);

typedef struct {
    uint32_t srcIP;         /* network order, as address_toNetworkIP */
    uint32_t dstIP;
    uint32_t payloadLength; /* packet_getPayloadLength: 0 = control packet, never dropped */
    uint32_t rngState;      /* sender host's rand_r state BEFORE the draw */
    uint64_t now;           /* worker clock at emit, ns */
} TopoPacketIn;

typedef struct {
    uint64_t time;          /* delivery event time, ns (0 if dropped) */
    uint32_t rngState;      /* sender's rand_r state after the draw */
    uint8_t delivered;      /* PDS_INET_SENT (1) / PDS_INET_DROPPED (0) */
    uint8_t _pad[3];
} TopoPacketOut;

/* worker_schedulePacket (shd-worker.c:332-370) for n packets of one scheduler window, host
 * buffers (includes the PCIe copies).  jumpNs/clampInterHost: shd-worker.c:310-324.  In lazy
 * mode every packet is answered as the reference's getReliability/getLatency calls would have
 * been in array (= emission) order: first-rooted-wins orientation and running-minimum pushes.
 * The caller captures in[i].rngState before the sender's draw and advances the sender's
 * Random by that one draw itself (tests/c/engine_window.c shows the engine-side adapter).
 * A packet whose address is not attached is not routed (the reference's getters return -1.0
 * for it, shd-topology.c:882-892): delivered 0, time 0, rngState after its draw; the others are
 * routed.  Returns 0 when every packet was routed, else the number of packets that were not, or
 * a negative error (the outputs are then undefined). */
int topology_routePacketBatch(Topology* top, const TopoPacketIn* in, TopoPacketOut* out, size_t n,
                              uint64_t jumpNs, int clampInterHost);

/* ---------------- Part 3: device-level boundary / library extras ---------------- */
int shdtopo_version(void);
/* CDATA topologies (shd-load-topology.c:57-82) without the temp file */
Topology* shdtopo_new_from_buffer(const char* graphml, size_t len);

/* options: "abort_on_error" (1), "lazy" (1 = K3 first-rooted-wins emulation, 0 = eager
 * forward rows), "delta" (delta-stepping bucket width, ms; default the mean edge latency),
 * "h0_phase" (where the landmark h0 sits in its bucket, [0, 1); default: at its bucket's end, a
 * gap of min(1 % of delta, half the smallest edge latency) below it; < 0: the round-4 bucket
 * shifts), "slots" (concurrent SSSP
 * workgroups), "device" (HIP device ordinal), "lds_hubs" (cap on LDS-resident hub distances,
 * -1 = fill), "par_hubs" (hubs with SSSP parent hints), "row_scan_chunk" (parent-pass pairs
 * per row-scan chunk, 64..2^20, default 16384: 16 B x batch of workspace per pair), "wg_per_cu" (SSSP workgroups sharing a
 * CU's LDS), "far_cap" / "near_cap" (entries per window bucket and overflow pile / per near
 * queue, 0 = sized from V; small values force the scanning fallback), "events" (1 = diagnostic
 * kernel with event counters), "tie_replay" (1: rows whose target chains cross a d-tied parent
 * are recomputed by the exact heap replay; 0: reported only), "replay_all" (test hook: every row
 * through the replay), "replay_slots" (concurrent replay wavefronts, 0 = auto), "replay_landmark"
 * (1: the replay skips relaxations into vertices a landmark bound proves popped),
 * "replay_int_keys" (1: u32 heap keys when every latency is an integer and V x max latency
 * < 2^32 - 1 -- exact; 0: always f64 keys), "tie_dense"
 * (-1 auto / 0 / 1: every row through the replay, no batch kernel, once a build replayed >= 90 %
 * of its rows or, on integer latencies, a 64-row probe before the first batched build found
 * >= 90 % of its rows crossing a tie), "devices" (N:
 * the table is built by N GPUs of this process -- rows sharded, RCCL all-gather of the rows and
 * all-reduce(MIN) of the minimum; devices device..device+N-1), "rccl" (1: use that exchange even
 * with one device), "batch" (sources per SSSP workgroup: 8; 2 / 4 / 16; any other value is
 * rejected), "batch_fill" (sources per batch, <= batch; 0 = auto: the fewest that finish the rows
 * in the same rounds of the slots), "source_order" / "batch_order" (row grouping and batch
 * dequeue order), "target_skip" (1: the batch relaxation drops pairs into
 * non-target vertices that would relax nothing reaching a target), "target_kappa" (iterations of
 * the target-aware kappa fixpoint behind that test, 0 = the row's smallest kappa; default 6),
 * "share" (1: a batched launch's workgroups that run out of batches take part in the running
 * batches' parent walks and epilogues -- the help board; 0, the default: each batch stays in its
 * workgroup and the board-less kernel runs; -1: the board for a launch whose batches fit one
 * round of the slots), "balance" (1, the default: from the second batched build of a graph on,
 * batches are sized (one round of the slots) or dequeued longest first (several rounds) by the
 * sources' costs measured from the earlier builds' batch times; 0: the grouping order only).
 * Returns 0 or -1 for an unknown key / bad value. */
int shdtopo_set_option(Topology* top, const char* key, double value);

/* attach by raw IP and a rand_r state (same algorithm and RNG use as topology_attach) */
int32_t shdtopo_attach_ip(Topology* top, uint32_t ip, uint32_t* rngState, const char* ipHint,
                          const char* geocodeHint, const char* typeHint, uint64_t* bwDownOut,
                          uint64_t* bwUpOut);
/* topology_detach by raw IP (shd-topology.c:1190-1197: the mapping goes, cached paths stay) */
void shdtopo_detach_ip(Topology* top, uint32_t ip);
double shdtopo_get_latency_ip(Topology* top, uint32_t srcIP, uint32_t dstIP);
double shdtopo_get_reliability_ip(Topology* top, uint32_t srcIP, uint32_t dstIP);

/* graph facts */
int64_t shdtopo_num_vertices(Topology* top);
int64_t shdtopo_num_edges(Topology* top);
int shdtopo_is_complete(Topology* top);
int shdtopo_is_directed(Topology* top);

/* attached-vertex table geometry: A distinct attached vertices, ascending vertex index */
int64_t shdtopo_num_attached(Topology* top);
int64_t shdtopo_attached_vertices(Topology* top, int32_t* out, int64_t cap);
int32_t shdtopo_column_of_ip(Topology* top, uint32_t ip);          /* -1 if unattached */
int32_t shdtopo_vertex_of_ip(Topology* top, uint32_t ip);          /* -1 if unattached */

/* Build the whole A x A table on this process's GPU(s) (SSSP or complete-pair kernel). */
int shdtopo_build(Topology* top);
/* Row shard [*r0, *r1) of device d out of n for A rows: ceil(A / n) rows each, the last shards
 * possibly short or empty (the split of option "devices" and of shadow_amd.sharding). */
void shdtopo_shard_rows(int64_t A, int n, int d, int64_t* r0, int64_t* r1);
/* Build rows [row0,row1) into caller-owned HBM: lr = {f64 lat, f64 rel}[rows][A],
 * hops = u16[rows][A], rowmin = f64[rows] (may be NULL).  Enqueued on `stream`. */
int shdtopo_build_rows(Topology* top, int64_t row0, int64_t row1, void* d_lr, void* d_hops,
                       void* d_rowmin, void* stream);
/* Install an assembled A x A table (e.g. after an RCCL all-gather) as the routing table.
 * The library copies it into its own buffers (same device). */
int shdtopo_bind_table(Topology* top, const void* d_lr, const void* d_hops, double globalMin,
                       void* stream);
/* Install an assembled table in place: the library reads the caller's buffers (same device; they
 * must stay valid and unchanged until the next build or bind) instead of copying 1.8 GB. */
int shdtopo_bind_table_ref(Topology* top, const void* d_lr, const void* d_hops, double globalMin,
                           void* stream);
/* Rebuild the whole table now for the current attached set (topology_getLatency & co. build it
 * lazily; this forces the build, e.g. to time it). */
int shdtopo_rebuild(Topology* top);
/* Copy the current table to host memory (lat, rel: f64[A*A]; hops: u16[A*A]; any may be NULL) */
int shdtopo_table_to_host(Topology* top, double* lat, double* rel, uint16_t* hops);

/* topology_routePacketBatch with the packets' vertices instead of their IPs (SoA host arrays;
 * -1 = not attached): the window adapter resolves them at emit, so a host detached before the
 * flush (the reference routed its packet at emit, shd-worker.c:345-369) is still routed while its
 * vertex is a table column.  Same outputs and return value. */
int shdtopo_route_batch_vertices(Topology* top, const int32_t* srcVertex, const int32_t* dstVertex,
                                 const uint32_t* payloadLength, const uint32_t* rngState,
                                 const uint64_t* now, size_t n, uint64_t jumpNs,
                                 int clampInterHost, TopoPacketOut* out);
/* Window bookkeeping of the engine-side adapter (include/shd_topology_window.h): while at least
 * one window is registered (hold +1 at topowindow_new, -1 at topowindow_free), a vertex that
 * loses its last host keeps its table column until shdtopo_window_release (called by every
 * flush after it routed), so the packets it emitted in the window are routed as the reference
 * routed them at emit.  Returns 0, -1 on a NULL topology. */
int shdtopo_window_hold(Topology* top, int delta);
int shdtopo_window_release(Topology* top);

/* Route n packets whose inputs are resident in HBM (SoA, attached-column indices). */
int shdtopo_route_batch_device(Topology* top, const int32_t* d_srcCol, const int32_t* d_dstCol,
                               const uint32_t* d_payload, const uint32_t* d_stateIn,
                               const uint64_t* d_now, int64_t n, uint64_t jumpNs, int clamp,
                               uint64_t* d_time, uint32_t* d_stateOut, uint8_t* d_delivered,
                               void* stream);

/* The same on device slot `slot` of a multi-GPU Topology (option "devices": every slot holds the
 * whole table after the exchange; inputs and outputs in that device's HBM, stream NULL = the
 * slot's own).  Slot 0 = shdtopo_route_batch_device. */
int shdtopo_route_batch_device_slot(Topology* top, int slot, const int32_t* d_srcCol,
                                    const int32_t* d_dstCol, const uint32_t* d_payload,
                                    const uint32_t* d_stateIn, const uint64_t* d_now, int64_t n,
                                    uint64_t jumpNs, int clamp, uint64_t* d_time,
                                    uint32_t* d_stateOut, uint8_t* d_delivered, void* stream);

/* lazily tracked minimum (reference trajectory, shd-topology.c:500-511) */
double shdtopo_get_lazy_minimum_latency(Topology* top);

/* Test hook: the source rows the lazy emulation has materialised so far (the rows whose
 * computeSourcePaths the reference would have run, shd-topology.c:900-915): up to cap vertices
 * with, per vertex, the attach epoch of its latest materialisation (epochs grow; a row
 * materialised again after a late attach gets a larger one) and the row minimum that
 * materialisation offered to the running minimum (shd-topology.c:500-511).  Any array may be
 * NULL.  Returns the number of materialised rows (may exceed cap), -1 on a NULL topology. */
int64_t shdtopo_lazy_rows(Topology* top, int32_t* vertex, uint64_t* epoch, double* rowmin,
                          int64_t cap);

typedef struct {
    double build_ms;          /* wall time of the last table build (device, event timed) */
    double sssp_kernel_ms;    /* event-timed duration of the last SSSP / pair kernel launch */
    double route_kernel_ms;   /* event-timed duration of the last packet-route launch */
    int64_t sources;          /* rows computed by the last build */
    int64_t targets;          /* A */
    int64_t ambiguous_pairs;  /* pairs whose path crosses a d-tied parent (heap order decides) */
    int64_t relaxations;      /* edge relaxations attempted by the last SSSP launch */
    int64_t long_paths;       /* pairs with more hops than the in-register path buffer */
    int64_t errors;           /* pairs with a missing edge (no self loop etc.) */
    double phase_ms[4];       /* SSSP kernel time summed over workgroups: init, near-far SSSP,
                                 parent derivation, per-target epilogue */
    int64_t near_iterations;  /* near-phase iterations summed over sources */
    int64_t far_splits;       /* buckets taken from the bucket window, summed over sources */
    int64_t slots;            /* concurrent SSSP workgroups of the last launch */
    int64_t events[8];        /* queue entries expanded, tail relaxations, tail improvements,
                                 window entries taken, overflow entries refilled, parent-pass
                                 vertices, relaxations onto settled tail vertices, stale
                                 entries skipped (events 1, 2, 6, 7 need option "events") */
    int64_t far_scan_sources; /* sources that overflowed a queue (scanning buckets instead) */
    double split_ms;          /* bucket changes + refills, summed over workgroups (in phase 1) */
    int64_t batch;            /* sources per SSSP workgroup of the last build (0: complete graph) */
    int64_t lds_hubs;         /* LDS-resident hub rows of the last SSSP launch */
    int64_t replay_rows;      /* rows recomputed by the exact igraph heap replay (rows with a
                                 d-tied parent on a target chain; every row of a directed graph) */
    double replay_ms;         /* event-timed duration of the heap-replay launch */
    int64_t replay_pops;      /* heap operations of the replay, summed over its rows: pops, */
    int64_t replay_pushes;    /*   pushes (first reach) and */
    int64_t replay_modifies;  /*   modifies (strict improvement of a queued vertex) */
    int64_t replay_slots;     /* concurrent replay wavefronts of the last launch */
    int64_t route_bad_packets; /* packets with a column outside [0, A), not routed (delivered 0,
                                  time 0, state unchanged), since the last table build */
    int64_t devices;          /* GPUs that built the last table (option "devices") */
    double exchange_ms;       /* RCCL all-gather + all-reduce(min) of that build (wall) */
    double parent_phase_ms[4]; /* batch kernel parent pass, summed over workgroups: walks, merged
                                  row scans, recount + finalize, next level */
    int64_t replay_lines[6];  /* profiling builds (-DSHD_RP_LINES=1) only, else 0: 64-B lines the
                                 replay touched in HBM -- sink loads, sink stores, shift-up loads,
                                 shift-up stores, relaxation loads, relaxation stores */
    int64_t batch_fill;       /* sources per batch of the last batched build (<= batch) */
    double replay_phase_ms[4]; /* profiling builds (-DSHD_RP_TIME=1) only, else 0: replay wall
                                  time summed over wavefronts -- sink, row + record loads, heap
                                  operations of the relaxation, init + epilogue */
    int64_t replay_sink_rounds; /* same builds: sink round trips and heap size, summed over pops, */
    int64_t replay_heap_sum;
    double replay_sink_ms[3];   /*   the sink's LDS walk, HBM rounds and moves, */
    int64_t replay_pf_hits;     /*   pops whose row bounds were prefetched */
    int64_t replay_skips;       /* replay relaxations into vertices the landmark bound proves
                                   popped (their vertex record is not read) */
    int64_t tie_dense;          /* 1: the last build ran every row through the replay because the
                                   topology is tie-dense (option "tie_dense") */
    double batch_wave_ms[6];    /* profiling builds (-DSHD_BATCH_TIME=1) only, else 0: batch
                                   kernel wave time summed over waves -- tail iterations' chunk
                                   loads, phase A, phase B, then the same for hub iterations */
    int64_t batch_rounds;       /*   phase-B rounds and the (edge, source) pairs that reached phase B */
    int64_t batch_edges_b;
    int64_t target_kappa_iters; /* iterations of the target-aware kappa fixpoint of the last target
                                   set (option "target_kappa") */
    double target_prep_ms;      /* wall time of that target-set preparation (target bits + kappa
                                   fixpoint in the relaxation copy; once per target set) */
    /* cold-build breakdown (the once-per-topology work a Shadow run pays before its first table,
       shd-topology.c:757-794 times the reference's equivalent inside the run): */
    double csr_ms;              /* wall time of the graph preparation (upload, relabel, CSR, h0
                                   distances, kappa-sorted copy); 0 when it ran in an earlier build */
    double csr_host_ms;         /*   of which CPU work on the host (not waiting for the GPU) */
    double csr_copy_ms;         /*   of which host <-> device copies (the parsed edge arrays in,
                                     perm / inv / pi / h0-tree parents out) */
    int64_t csr_h0_rounds;      /*   frontier rounds of its h0 distances (pi = d(h0, .)) */
    double order_ms;            /* host: source order, batch order and bucket shifts of the last
                                   batched build */
    double replay_prep_ms;      /* wall time of the heap replay's incidence CSR (once per topology) */
    int64_t touched_lines;      /* tail distance lines the batches of the last build reset (only the
                                   lines a batch lowered from +inf are reset for the next one) */
    int64_t csr_host_runs;      /* host-side graph preparations in the last build (a multi-GPU
                                   build prepares once and shares it with its peer engines) */
    double workspace_ms;        /* wall time of allocating + initialising the SSSP workspace
                                   (first build, or a layout change) */
    double csr_step_ms[8];      /* graph preparation steps (wall): upload of the parsed edges,
                                   degrees + relabel, adjacency rows, h0 distances, h0 tree +
                                   record fields, kappa-sorted copy, host copies out, (unused) */
    double module_load_ms;      /* device init: loading the kernels' code objects and the first
                                   segmented sort's host setup (once per engine, before its
                                   first build) */
    double build_wall_ms;       /* wall time of the last whole-table build (topology_getLatency's
                                   lazy build, shdtopo_build / shdtopo_rebuild) */
    int64_t walk_steps;         /* parent-pass walk steps (pairs resolved) of the last build */
    double build_step_ms[8];    /* wall checkpoints of the last whole-table build: device init,
                                   geometry + table buffers, preparation up to the SSSP launch
                                   (graph, workspace, target set, order), the SSSP kernel, the tie
                                   replay + rest of the rows, statistics, (unused) x 2 */
    int64_t exchange_kind;      /* the last build's row exchange (option "exchange"): 0 none (one
                                   device), 1 RCCL all-gather + all-reduce(MIN) after every shard,
                                   2 push: each shard copied into the other devices' tables (peer
                                   DMA) as soon as it is done (engines sharing a device, RCCL
                                   unavailable, or exchange = 2) */
    int64_t walk_kinds[4];      /* of the walk steps: parents certified by the h0-tree guess, by a
                                   tail's recorded improver, by a hub's recorded improver, and pairs
                                   sent to the merged row scans */
    double build_wait_ms;       /* the last whole-table build's wait for the build lock (the
                                   attach-time preparation thread, or another builder) */
    double attach_prep_ms;      /* wall time of the attach-time preparation (option
                                   "prepare_on_attach": device init + graph preparation in a
                                   background thread from the first attach on, overlapping the
                                   host's attach phase; 0 if it did not run) */
    int64_t replay_int_keys;    /* 1: the last replay ran on u32 heap keys (every latency an
                                   integer, V x max latency < 2^32 - 1: exact), 0: f64 keys */
    int64_t tie_probe_rows;     /* the last build's tie probe (integer latencies, before the first
                                   batched build): sample rows run through the batch kernel, */
    int64_t tie_probe_flagged;  /*   of which crossing a d-tied parent (>= 90 %: tie-dense, every
                                     row goes straight to the heap replay) */
    double tie_probe_ms;        /*   and its wall time */
    double first_attach_to_table_ms; /* wall time from the first attach to the first table
                                        installed (once per topology; 0 before) */
    int64_t exchange_bytes;     /* bytes each device received in the last row exchange (all-gather
                                   of the other devices' rows, hops and row minima) */
    int64_t csr_host_runs_total; /* host-side graph preparations since the topology was loaded,
                                    the owner's and every peer engine's, the attach-time
                                    preparation thread's included */
    int64_t sweep_events[4];    /* profiling builds (-DSHD_BATCH_TIME=1) only, else 0: the batch
                                   kernel's phase-B rounds holding a tail-target pair, tail-target
                                   pairs, hub-target pairs, (unused) */
    int64_t write_lines[16];    /* profiling builds (-DSHD_BATCH_WRCOUNT=1) only, else 0: 64-B lines
                                   the batch kernel's stores and atomics touched, by category
                                   (topo_sssp_batch.hip WL_*): relaxation atomicMin, tie tags,
                                   improver hints, pending atomics, touched atomics, near-mask
                                   atomics; mask stores; pending words; line reset; touched-word
                                   clears; pair records; parent scratch; table output; hub rows and
                                   hints; queue appends; other */
    int64_t read_lines[8];      /* the same builds: 64-B lines read, by category (RL_*): phase-B
                                   pre-checks, phase-A records, chunk loads, sweeps, parent walks,
                                   epilogue, reset, other (hint pass, row scans) */
    double attach_prep_step_ms[4]; /* the attach-time preparation's parts (wall): device init (HIP
                                      queues, code objects), graph preparation, edge scan, the
                                      batched SSSP's workspace (allocation + initialisation) */
    int64_t pair_matrix_builds; /* complete topologies: times the resident A x A direct-edge
                                   matrices were (re)built (once per attached set; cumulative) */
    double device_kernel_ms[8]; /* the last multi-device build (option "devices"), per device slot
                                   (first 8): event time of its row shard's kernels (SSSP or pair
                                   kernel, + heap replay), */
    double device_build_ms[8];  /*   wall time of its row shard's build, */
    int64_t device_rows[8];     /*   and its rows */
    int64_t dev_inits;          /* device initialisations of this topology (HIP stream, events, code
                                   objects): 1, or 2 when the "device" option moved it */
    double init_bg_ms;          /* wall time of topology_new's background device init (overlaps the
                                   GraphML parse; 0 if it did not run) */
    double path_seconds_total;  /* shortestPathTotalTime of the reference (shd-topology.c:792): wall
                                   seconds of every table / row build so far */
    int64_t paths_computed;     /* shortestPathCount (shd-topology.c:793): source rows built so far;
                                   both are logged at topology_free (:445-446) */
    int64_t batch_layout_measured; /* 1: the last batched launch used the measured layout (option
                                      "balance": batches sized / ordered by the sources' costs
                                      from earlier builds' batch times), 0: the grouping order */
    int64_t batches;            /*   batches of that launch */
    int64_t rows_to_host;       /* getters (topology_getLatency & co.): table rows copied to the
                                   host on their first read, cumulative (16 A bytes each; the
                                   getters never copy the whole A x A table) */
    double rows_to_host_ms;     /*   and the wall time of those copies */
    int64_t prep_trigger;       /* what started the background graph preparation (attach_prep_ms):
                                   0 none, 1 the first attach, 2 topology_new (right after the
                                   parse; SHDTOPO_NO_LOAD_PREP=1 turns that off) */
    double exchange_exposed_ms; /* the last multi-device build: wall time from the last shard's
                                   rows to the end of the exchange (the part of exchange_ms no
                                   kernel hid; exchange_kind 2 overlaps the slower shards) */
    int64_t workspace_bytes;    /* HBM held by the batched SSSP's workspace (all slots) */
} ShdStats;
int shdtopo_get_stats(Topology* top, ShdStats* out);

/* Test hook: the measured batch layout (option "balance") for per-position
 * costs cost[rows] (grouping order) with a batch's fixed part `fixed`, batch fill `fill`, `slots`
 * workgroups and batch width `batch`.  order u32[rows] receives the grouping positions in launch
 * order, starts u32[rows + 1] the batch starts (*nbatches + 1 entries): one round of the slots =
 * runs of the grouping order minimising the largest predicted batch; several rounds = batches of
 * `fill` consecutive positions, longest predicted first, the ragged one last.  Returns 0, or -1
 * when no layout applies (the build then keeps the grouping order).  Host-only: no device use. */
int shdtopo_test_batch_layout(const double* cost, int64_t rows, double fixed, int fill, int slots,
                              int batch, uint32_t* order, uint32_t* starts, int64_t* nbatches);

/* Test hook: the segmented sort of the target-aware re-sort on HIP device 0 -- nseg rows
 * (rowptr u32[nseg + 1] over n f32 keys) each sorted ascending and stably; keys_out receives the
 * sorted keys, idx_out their input positions.  reference = 1 runs the whole-adjacency hipcub
 * segmented radix sort the library's kernels replace (the order they must reproduce).  Returns 0,
 * -1 on bad arguments, or a HIP error. */
int shdtopo_test_segsort(const uint32_t* rowptr, int64_t nseg, const float* keys, int64_t n,
                         int reference, float* keys_out, uint32_t* idx_out);

/* Test hook: run the exact heap replay (igraph_get_shortest_paths_dijkstra restated on the GPU)
 * from vertex `src` over the current attached set.  full = 1 runs to an empty heap instead of
 * stopping when every attached vertex is popped.  dist f64[V] (-1 = unreached) and parent int32[V]
 * (-1 = none) receive the replay's result in original vertex ids.  Returns 0 or an error. */
int shdtopo_replay_source(Topology* top, int32_t src, int full, double* dist, int32_t* parent);

/* Test hook: the device graph preparation (topo_prep.hip) read back -- perm
 * int32[V] (relabelled -> original vertex), rowptr u32[V+1], the adjacency columns u32[2E']
 * (relabelled ids, rows ascending by neighbour), pi f64[V] (= d(h0, .), relabelled ids) and the
 * h0-tree parents u32[V] (relabelled, ~0 = none).  Any pointer may be NULL (call with NULLs to
 * size col).  Prepares the graph if needed.  Returns 2E', or a negative error (-2: complete or
 * directed topology, which have no such CSR). */
int64_t shdtopo_export_csr(Topology* top, int32_t* perm, uint32_t* rowptr, uint32_t* col,
                           double* pot, uint32_t* treeParent);

/* Copy the parsed graph into host arrays (document order; any pointer may be NULL):
 * eu, ev int32[E]; elat, eloss f64[E]; vloss f64[V].  Used by tools and oracle cross-checks. */
int shdtopo_export_graph(Topology* top, int32_t* eu, int32_t* ev, double* elat, double* eloss,
                         double* vloss);

/* Write the loaded graph back out as GraphML (same key schema as the bundled resource files). */
int shdtopo_write_graphml(Topology* top, const char* path);

/* ---- synthetic workloads (BASELINE.json configs 4/5; tools, not on the routing path) ---- */
typedef struct {
    uint64_t seed;
    int64_t n_routers;   /* 990000 */
    int64_t n_poi;       /* 10000 */
    int64_t n_edges;     /* 10000000 undirected edges in total, incl. poi uplinks + self loops */
    int integer_latency; /* 1: latency ~ U{1..100} (heavy ties) */
    double alpha;        /* Chung-Lu endpoint weight ~ rank^(-alpha); 1/1.1 */
    int directed;        /* 1: a directed topology -- every non-loop edge becomes two arcs, the
                            reverse one with its own latency and loss draw (uplinks 5.0 both
                            ways), so E = 2 x n_edges - n_poi (tools: directed-path probes) */
} ShdSynthParams;
Topology* shdtopo_new_synthetic(const ShdSynthParams* p);

/* Attach n_hosts hosts with Tor-like type hints (94 % client, 5 % relay, 1 % server) following
 * Shadow's seed chain (master --seed -> slave seed -> per-host nodeSeed), IPs
 * 11.0.0.1 + k; host k < (number of poi with a usable ip) is pinned to the k-th poi by an exact
 * ipHint (so every poi of a synthetic topology is attached); then emit n_packets packets of one window: src uniform over hosts, dst by role,
 * payload 1448 w.p. 0.8 else 0, pre-draw rand_r state from each host's stream, now ~
 * U[t0, t0 + jump).  Output arrays are host memory of length n_packets (hostState: n_hosts,
 * the hosts' states after attach). */
int shdtopo_synth_packets(Topology* top, uint64_t seed, int64_t n_hosts, int64_t n_packets,
                          uint64_t t0, uint64_t jump, int32_t* srcCol, int32_t* dstCol,
                          uint32_t* payload, uint32_t* stateIn, uint64_t* now,
                          uint32_t* srcIP, uint32_t* dstIP);

#ifdef __cplusplus
}
#endif
#endif /* SHD_TOPOLOGY_ABI_H_ */
