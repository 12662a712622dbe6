#!/usr/bin/env python3
"""bench.py -- routing-table build GTEPS + packet-routes/s on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE.json configs 4 + 5; synthetic, generated in memory):
  * C4: power-law Internet topology, 990,000 routers + 10,000 poi, exactly 10,000,000 undirected
    edges (Chung-Lu, deduplicated, spanning path, poi uplinks + self loops), seed 20261015,
    written as GraphML and loaded back through topology_new;
  * C5: 100,000 Tor-like hosts attached by type hint (94/5/1 % client/relay/server) through
    Shadow's seed chain; one scheduler window of 10,000,000 packets.
A step = one build of the whole attached-vertex routing table (all A = 10^4 sources x A targets:
batched SSSP + parents + epilogue per source, rows sharded over the GPUs, the row exchange and the
runahead minimum, the table installed in the library).
value = A * E / t_step / 1e9 (Graph500 SSSP convention, undirected E) = GTEPS, whole job.
cold_build = the first build of the loaded topology -- graph preparation (CSR, relabel, h0
distances, kappa copy), target preparation, kernels, exchange -- what a Shadow run pays once.
Packet routes are timed separately over resident windows and reported as packet_routes_per_s.

Multi-GPU.  Default --mode library: the process that owns the Topology drives N
GPUs itself (option "devices", RCCL all-gather + all-reduce(MIN) inside the library), as one
Shadow process would.  Under torchrun only rank 0 works in this mode; the other ranks wait.
--mode torchrun: one process per GPU builds its row shard and torch.distributed (RCCL) exchanges.

Launch: python bench.py [--gpus N --steps K --warmup W]   (N GPUs from one process), or
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import shadow_amd as sa  # noqa: E402
from shadow_amd import sharding  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
SEED = 20261015
PROFILE_TAG = "r06e"           # profiles/<tag>_*_pmc.json: the committed counter passes


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def source_hash():
    """Hash of the engine's sources: a committed PMC file applies only to the code it measured."""
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(ROOT, "shadow_amd", "csrc", "*"))):
        if p.endswith((".hip", ".cpp", ".h")):
            h.update(open(p, "rb").read())
    return h.hexdigest()[:12]


def cpu_share():
    """CPU threads this job may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU box
    exports 16 per GPU; os.cpu_count() there is the whole machine's count)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(top, attached, n_sample, n_sample_mt, nthreads_mt):
    """The reference path's CPU restatement (oracle: igraph-0.7 binary-heap Dijkstra + helper),
    timed on this host on bounded samples of sources (BASELINE.md's plan: 64 sources): 1 thread
    (the reference's concurrency: Dijkstra runs under the global graphLock) and
    every thread of the job's CPU share (sources are independent).  The sample's own rate is
    `value`; the linear extrapolation to the full table is reported apart from it."""
    import oracle
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    t0 = time.time()
    g = oracle.OGraph(V, eu, ev, elat, eloss, vloss)
    t_setup = time.time() - t0
    E, A = len(eu), len(attached)
    srcs = attached[:n_sample]
    t0 = time.time()
    g.source_rows(srcs, attached, nthreads=1)
    t = time.time() - t0
    out = dict(value=len(srcs) * E / t / 1e9, unit="GTEPS", cores=1, kind="port",
               sample="%d of %d sources x %d targets (Dijkstra + per-target helper) on 1 thread: "
                      "%.1f s measured" % (len(srcs), A, A, t),
               sample_sources=len(srcs), sample_s=round(t, 2),
               extrapolated=dict(full_table_s=round(t / len(srcs) * A, 1),
                                 note="linear in the source count (%d sources)" % A),
               seconds_per_source=t / len(srcs), oracle_setup_s=t_setup)
    if n_sample_mt > 0 and nthreads_mt > 1:
        srcs = attached[n_sample:n_sample + n_sample_mt]
        t0 = time.time()
        g.source_rows(srcs, attached, nthreads=nthreads_mt)
        t = time.time() - t0
        out["all_cores"] = dict(
            value=len(srcs) * E / t / 1e9, unit="GTEPS", cores=nthreads_mt,
            sample="%d sources x %d targets on %d threads (the job's CPU share): %.1f s measured"
                   % (len(srcs), A, nthreads_mt, t),
            sample_sources=len(srcs), sample_s=round(t, 2),
            extrapolated=dict(full_table_s=round(t / len(srcs) * A, 1),
                              note="linear in the source count"),
            seconds_per_source=t / len(srcs))
    return out


def _chunks(n, k):
    b = [n * i // k for i in range(k + 1)]
    return [(b[i], b[i + 1]) for i in range(k) if b[i + 1] > b[i]]


def parallel_calls(fn, n, nthreads):
    """fn(lo, hi) over nthreads contiguous chunks of [0, n) in threads (the oracle's ctypes calls
    release the GIL, so the chunks run on separate cores)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=nthreads) as ex:
        return list(ex.map(lambda c: fn(*c), _chunks(n, nthreads)))


def directed_line(hosts, steps=3):
    """C4-dir: the C4 generator with every non-loop edge as two arcs of independent latency
    (1M vertices, 19.99M arcs; igraph mode OUT, shd-topology.c:153,762-763), its whole attached
    table built through the batch kernel (out-rows relaxed, parents from the in-rows).  Not a
    BASELINE config: it shows the directed path at the bench's size (round 4 sent every directed
    row through the heap replay: ~22.9 s for this table, profiles/r05k_directed_probe.log)."""
    t0 = time.time()
    dtop = sa.Topology.synthetic(seed=SEED, directed=True)
    gen_s = time.time() - t0
    dtop.synth_packets(SEED, hosts, 0, 10**9, 10**7)
    A, E = len(dtop.attached_vertices()), dtop.num_edges
    ms, kms = [], []
    for i in range(1 + steps):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        dtop.rebuild()
        torch.cuda.synchronize()
        if i > 0:  # the first build prepares the graph (cold)
            ms.append((time.perf_counter() - t1) * 1e3)
            kms.append(dtop.stats()["sssp_kernel_ms"])
    st = dtop.stats()
    t = float(np.mean(ms)) / 1e3
    out = dict(workload="C4-dir: C4 with every non-loop edge as two arcs of independent latency "
                        "(directed, mode OUT), all %d x %d attached pairs" % (A, A),
               vertices=dtop.num_vertices, arcs=E, generate_s=round(gen_s, 2), steps=steps,
               ms_per_build=round(t * 1e3, 2), kernel_ms=round(float(np.mean(kms)), 3),
               gteps=round(A * E / t / 1e9, 3), replay_rows=st["replay_rows"],
               ambiguous_pairs=st["ambiguous_pairs"], errors=st["errors"],
               min_latency_ms=dtop.getMinimumLatency())
    dtop.free()
    return out


def complete_table_lines(repeats=20, nthreads=1, devices=1, cpu=True):
    """BASELINE configs 2 (plab, 303 x 303, "on 1 MI355X") and 3 (full Internet, 183 x 183, "on 8
    MI355X"): the complete-graph pair table (_topology_lookupPath for every attached pair,
    shd-topology.c:835-873) built by shdtopo_rebuild -- the whole-table build Shadow's first
    getter triggers: on `devices` GPUs the rows are sharded over the library's engines and
    exchanged (RCCL all-gather + all-reduce(MIN)).  One host per vertex via its unique geocode
    hint.  Reported: the build call's wall time (build_ms), the pair kernel's
    event time (kernel_ms: the slowest device's), per device its shard kernel and rows, and the
    exchange; 34 B per pair (roofline of pair_table_complete_kernel).  CPU: the oracle's
    restatement on one thread and on every thread of the job's share (N = 1 runs only)."""
    import lzma
    import oracle
    out = {}
    for cfg, name in (("C2", "topology.plab"), ("C3", "topology")):
        path = os.path.join(ROOT, "tests", "golden", "resource", name + ".graphml.xml.xz")
        with lzma.open(path) as f:
            data = f.read()
        top = sa.Topology.from_buffer(data)
        g = oracle.OGraph.from_graphml(data)
        if devices > 1:
            top.set_option("devices", devices)
        geos = list(g.vattrs["geocode"])
        st = 1
        for k, geo in enumerate(geos):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            top.attach_ip(sa.ip_to_network("11.%d.%d.%d" % (k >> 16, (k >> 8) & 255, k & 255)),
                          st, geocodeHint=geo)
        A = len(top.attached_vertices())
        ms, wall, dk, xm = [], [], [], []
        for i in range(repeats + 2):
            top.rebuild()
            s_ = top.stats()
            if i >= 2:
                ms.append(s_["sssp_kernel_ms"])
                wall.append(s_["build_wall_ms"])
                dk.append(s_["device_kernel_ms"][:max(1, min(8, devices))])
                xm.append(s_["exchange_ms"])
        k_ms = float(np.median(ms))
        pairs = A * A
        line = dict(topology=name, attached=A, pairs=pairs, devices=devices,
                    build_ms=round(float(np.median(wall)), 4), kernel_ms=round(k_ms, 4),
                    gpu_pairs_per_s=round(pairs / (float(np.median(wall)) / 1e3), 1),
                    kernel_pairs_per_s=round(pairs / (k_ms / 1e3), 1),
                    kernel="pair_table_complete_kernel (records, hops, row minima, global "
                           "minimum: one launch per device)",
                    pair_matrix_builds=int(s_["pair_matrix_builds"]),
                    roofline=dict(bound="hbm", bytes_per_unit=34, units_per_launch=pairs,
                                  achieved=round(pairs * 34 / (k_ms / 1e3) / 1e9, 2),
                                  peak=HBM_PEAK_GBS, unit="GB/s",
                                  frac=round(pairs * 34 / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5)),
                    note="launch-bound: %d pairs are a few microseconds of HBM time; the edge "
                         "matrices stay resident while the attached set is unchanged" % pairs)
        if devices > 1:
            line["device_kernel_ms"] = [round(float(x), 4) for x in np.median(np.asarray(dk), axis=0)]
            line["device_rows"] = list(s_["device_rows"][:min(8, devices)])
            line["exchange"] = dict(kind={0: "none", 1: "rccl", 2: "push"}.get(
                int(s_["exchange_kind"]), "?"), ms=round(float(np.median(xm)), 4),
                bytes_per_device=int(s_["exchange_bytes"]))
        if cpu:
            a = np.asarray(sorted(set(top.attached_vertices().tolist())), np.int32)
            S, D = np.meshgrid(a, a, indexing="ij")
            Sr, Dr = S.ravel(), D.ravel()
            t0 = time.perf_counter()
            g.complete_pairs(Sr, Dr)
            t_cpu = time.perf_counter() - t0
            t0 = time.perf_counter()
            parallel_calls(lambda lo, hi: g.complete_pairs(Sr[lo:hi], Dr[lo:hi]), len(Sr), nthreads)
            t_cpu_mt = time.perf_counter() - t0
            line.update(cpu_pairs_per_s=round(pairs / t_cpu, 1), cpu_cores=1,
                        cpu_all_cores=dict(pairs_per_s=round(pairs / t_cpu_mt, 1), cores=nthreads))
        top.free()
        out[cfg] = line
    return out


def cpu_route_baseline(lat, rel, payload, state, now, jump, nthreads=1):
    """worker_schedulePacket's restatement (oracle) over the whole window: packets/s."""
    import oracle
    t0 = time.perf_counter()
    parallel_calls(lambda lo, hi: oracle.route_packets(lat[lo:hi], rel[lo:hi], payload[lo:hi],
                                                       state[lo:hi], now[lo:hi], jump, 1),
                   len(lat), nthreads)
    return len(lat) / (time.perf_counter() - t0)


def getters_block(top, pk, n_q, nthreads, cpu):
    """The per-packet getter path as unchanged Shadow drives it: n_q queries of
    the C5 window, each the getReliability + getLatency pair of shd-worker.c:352,360, issued by
    worker threads through the C ABI (tests/c/libgetter_bench.so).  Pass 1 follows a rebuild: the
    lazy emulation materialises rows and each row the queries touch is copied to the host on its
    first read (16 A bytes).  Passes 2-3 are warm (1 thread, then every thread of the job's share).
    Beside it, on N = 1, the reference's own cached path restated in C (oracle.c orc_cache_*:
    virtualIP + two-level path cache behind RW locks, shd-topology.c:450-531,876-958), timed on
    cache hits only."""
    import ctypes
    g = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libgetter_bench.so"))
    P = ctypes.c_void_p
    g.getbench_run.restype = ctypes.c_int64
    g.getbench_run.argtypes = [P, ctypes.c_int64, P, P, ctypes.c_int, P, P]
    pp = lambda a: a.ctypes.data_as(P)
    sip = np.ascontiguousarray(pk["src_ip"][:n_q], np.uint32)
    dip = np.ascontiguousarray(pk["dst_ip"][:n_q], np.uint32)
    n = len(sip)
    calls = 2 * n

    def run(nt):
        lat, rel = np.empty(n), np.empty(n)
        ns = g.getbench_run(top._h, n, pp(sip), pp(dip), int(nt), pp(lat), pp(rel))
        if ns <= 0:
            raise RuntimeError("getter bench failed (%d)" % ns)
        return ns / 1e9, lat, rel

    s0 = top.stats()
    t0, lat0, rel0 = run(nthreads)
    s1 = top.stats()
    t1, lat1, rel1 = run(1)
    tn, latn, reln = run(nthreads)
    u = lambda a: a.view(np.uint64)
    # (the orientation of an answer depends on which rows the lazy emulation materialised first,
    # shd-topology.c:894-915, so passes may differ in the last bits of asymmetric pairs; the
    # getters' values are checked against the table by tests/test_getters_mt.py)
    valid = bool(all(np.all(x > 0) for x in (lat0, lat1, latn)) and
                 all(np.all((x >= 0) & (x <= 1)) for x in (rel0, rel1, reln)))
    out = dict(queries=n, getter_calls=calls, threads=nthreads,
               cold_pass=dict(threads=nthreads, ms=round(t0 * 1e3, 2),
                              rows_copied=int(s1["rows_to_host"] - s0["rows_to_host"]),
                              rows_copy_ms=round(s1["rows_to_host_ms"] - s0["rows_to_host_ms"], 2),
                              bytes_per_row=16 * len(top.attached_vertices())),
               ns_per_call_1_thread=round(t1 * 1e9 / calls, 1),
               ns_per_call_per_thread=round(tn * 1e9 * nthreads / calls, 1),
               calls_per_s_1_thread=round(calls / t1, 1),
               calls_per_s_all_threads=round(calls / tn, 1),
               answers_valid=valid,
               note="getter call = one topology_getReliability or topology_getLatency (Shadow "
                    "issues the pair per packet); the first pass after a rebuild copies each row "
                    "it reads once (rows_copied x bytes_per_row), later calls read host rows "
                    "without a lock")
    if cpu:
        import oracle
        ips = np.unique(np.concatenate([sip, dip]))
        verts = np.array([top.vertex_of_ip(int(x)) for x in ips], np.int32)
        vmap = dict(zip(ips.tolist(), verts.tolist()))
        sv = np.array([vmap[x] for x in sip.tolist()], np.int32)
        dv = np.array([vmap[x] for x in dip.tolist()], np.int32)
        oc = oracle.OracleCache(ips, verts, directed=top.is_directed)
        oc.store(sv, dv, lat1, rel1)
        r1, olat, orel = oc.bench(sip, dip, 1)
        rn, _, _ = oc.bench(sip, dip, nthreads)
        oc.free()
        out["reference_cached"] = dict(
            kind="port", ns_per_call_1_thread=round(r1 * 1e9 / calls, 1),
            ns_per_call_per_thread=round(rn * 1e9 * nthreads / calls, 1),
            calls_per_s_1_thread=round(calls / r1, 1),
            calls_per_s_all_threads=round(calls / rn, 1),
            answers_equal=bool(np.array_equal(u(olat), u(lat1)) and np.array_equal(u(orel), u(rel1))),
            note="the reference's getPathEntry on cache hits (the pairs filled beforehand): 2 "
                 "virtualIP lookups + 1-2 path-cache lookups, each under its RW lock")
    return out


def batched_model(st, pairs, k_ms, traffic):
    """roofline.model_batched: the bytes the batched, target-pruned SSSP
    moves per build as implemented, from the kernel's own counters of the measured build --
      * adjacency: every expansion reads its row bounds (8 B) and its kappa-cut row of 16-B
        relaxation records (events.expanded expansions, events.tail_relax records);
      * distance lines: every [V][K] tail line a batch touches is written once and reset once for
        the next batch (2 x 64 B per touched line; hub lines live in LDS);
      * output: 18 B per pair (lat, rel, hops).
    It assumes perfect reuse inside a batch (a line touched by many relaxations moves once), so it
    is a lower bound for this algorithm; counter traffic / model is its waste ratio.  The
    per-relaxation bound (one 64-B line per relaxation record) is reported beside it."""
    ev = st["events"]
    exp_, recs, touched = int(ev["expanded"]), int(ev["tail_relax"]), int(st["touched_lines"])
    comp = dict(adjacency=8 * exp_ + 16 * recs, distance_lines=128 * touched, output=18 * pairs)
    b = sum(comp.values())
    k_s = k_ms / 1e3
    out = dict(bytes=b, components=comp, expansions=exp_, relaxation_records=recs,
               touched_lines=touched,
               achieved=round(b / k_s / 1e9, 2) if k_s > 0 else None, unit="GB/s",
               frac=round(b / k_s / 1e9 / HBM_PEAK_GBS, 5) if k_s > 0 else None,
               traffic_over_model=round(traffic / b, 3) if (traffic and b) else None,
               per_relaxation_line_bytes=64 * recs,
               note="lower bound of the batched algorithm's bytes (perfect reuse within a batch); "
                    "traffic_over_model = the PMC bytes per launch over it (its waste ratio)")
    return out


def load_pmc(path, key):
    """A committed counter summary (tools/summarize_prof.py) if it was measured on this exact
    workload and code (key), else None."""
    if not path or not os.path.exists(path):
        return None
    try:
        pm = json.load(open(path))
    except Exception:
        return None
    return pm if pm.get("config_key") == key else None


def hbm_roofline(kernel, kernel_ms, traffic_pm, model_bytes_per_unit, units, model_note):
    """Roofline of one kernel: achieved = measured HBM bytes per launch (PMC, FETCH_SIZE +
    WRITE_SIZE in separate passes) / the launch time -- a rate the memory system actually
    delivered, so frac <= 1.  The algorithmic model of SURVEY.md 8(d) is reported beside it."""
    k_s = kernel_ms / 1e3
    traffic = traffic_pm["hbm_bytes_per_launch"] if traffic_pm else None
    achieved = traffic / k_s / 1e9 if (traffic and k_s > 0) else None
    model_achieved = units * model_bytes_per_unit / k_s / 1e9 if k_s > 0 else None
    out = dict(bound="hbm", kernel=kernel, kernel_ms=round(kernel_ms, 3),
               achieved=round(achieved, 2) if achieved else None, peak=HBM_PEAK_GBS, unit="GB/s",
               frac=round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
               traffic=traffic, units_per_launch=units,
               pmc=traffic_pm.get("source") if traffic_pm else "no counter pass for this code",
               model=dict(bytes_per_unit=model_bytes_per_unit,
                          achieved=round(model_achieved, 2) if model_achieved else None,
                          frac=round(model_achieved / HBM_PEAK_GBS, 5) if model_achieved else None,
                          note=model_note))
    if traffic_pm and traffic_pm.get("dram_requests_per_launch"):
        out["dram_requests_per_unit"] = round(traffic_pm["dram_requests_per_launch"] / max(1, units))
        out["dram_requests_per_s"] = round(traffic_pm["dram_requests_per_launch"] / k_s)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=("library", "torchrun"), default="library",
                    help="library: one process drives the GPUs (option devices); torchrun: one "
                         "process per GPU exchanging through torch.distributed")
    ap.add_argument("--routers", type=int, default=990_000)
    ap.add_argument("--poi", type=int, default=10_000)
    ap.add_argument("--edges", type=int, default=10_000_000)
    ap.add_argument("--hosts", type=int, default=100_000)
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--route-steps", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=64,
                    help="sources timed on 1 CPU thread (about 1 s each; BASELINE.md: 64)")
    ap.add_argument("--cpu-sample-mt", type=int, default=256,
                    help="sources timed on all threads of the job's CPU share")
    ap.add_argument("--no-graphml", action="store_true",
                    help="skip the GraphML write + topology_new load of the generated topology")
    ap.add_argument("--no-complete", action="store_true", help="skip the C2/C3 table lines")
    ap.add_argument("--no-directed", action="store_true", help="skip the C4-dir line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--getter-queries", type=int, default=1_000_000,
                    help="queries of the getters block (0: skip it)")
    ap.add_argument("--delta", type=float, default=0.0)
    ap.add_argument("--integer", action="store_true",
                    help="C4-int variant (integer latencies U{1..100}: heavy parent ties)")
    ap.add_argument("--batch", type=int, default=8, help="sources per SSSP workgroup (2/4/8/16)")
    ap.add_argument("--opt", action="append", default=[], help="key=value library option")
    ap.add_argument("--pmc-tag", default=PROFILE_TAG)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    library = args.mode == "library"
    ngpu = max(args.gpus, world) if library else world
    if world > 1:
        if library:
            # rank 0 drives every GPU through the library; the others only wait for it (gloo:
            # they never touch a GPU)
            dist.init_process_group("gloo")
            if rank != 0:
                dist.barrier()
                dist.destroy_process_group()
                return
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if not (world > 1 and not library):
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if library and ngpu > torch.cuda.device_count():
        raise SystemExit("--gpus %d > %d visible devices" % (ngpu, torch.cuda.device_count()))

    # ---- workload (generation and loading are outside the timed region).  The generated C4
    # topology is written as GraphML once and loaded back through topology_new
    # (shd-topology.c:1237 -> _topology_loadGraph :95-123), as Shadow loads it; the round trip
    # must reproduce the generator's graph bit for bit. ----
    t0 = time.time()
    gen = sa.Topology.synthetic(seed=SEED, n_routers=args.routers, n_poi=args.poi,
                                n_edges=args.edges, integer_latency=args.integer)
    graphml = dict(generate_s=round(time.time() - t0, 2))
    top = gen
    torchrun = world > 1 and not library
    if not args.no_graphml:
        import tempfile
        path = os.path.join(tempfile.gettempdir(), "shdtopo_c4_%s_%d.graphml.xml" % (
            "int" if args.integer else "real", os.getpid() if not torchrun else 0))
        if torchrun:
            path = path.replace("_0.graphml", "_%s.graphml" % os.environ.get("MASTER_PORT", "0"))
        try:
            if rank == 0:
                t1 = time.time()
                gen.write_graphml(path)
                graphml["write_s"] = round(time.time() - t1, 2)
                graphml["bytes"] = os.path.getsize(path)
            if torchrun:
                dist.barrier()
            t1 = time.time()
            top = sa.Topology.new(path)
            graphml["load_s"] = round(time.time() - t1, 2)
            assert top is not None, "topology_new failed on the written GraphML"
            a_, b_ = gen.export_graph(), top.export_graph()
            assert a_[0] == b_[0] and all(np.array_equal(np.asarray(x).view(np.uint8),
                                                         np.asarray(y).view(np.uint8))
                                          for x, y in zip(a_[1:], b_[1:])), "GraphML round trip"
            graphml["round_trip_bit_exact"] = True
        finally:
            if torchrun:
                dist.barrier()
            if rank == 0 and os.path.exists(path):
                os.unlink(path)
    del gen
    top.set_option("device", local)
    top.set_option("batch", args.batch)
    if args.delta:
        top.set_option("delta", args.delta)
    for kv in args.opt:
        k, v = kv.split("=")
        top.set_option(k, float(v))
    if library and ngpu > 1:
        top.set_option("devices", ngpu)
    window0 = 10_000_000  # Shadow's default 10 ms window until the runahead is known
    # ---- the attach phase (Shadow creates its hosts: topology_attach per host), timed as wall
    # clock; the first table is built right after it, as Shadow's first packet would trigger it,
    # so any part of the attach-time preparation the attaches do not hide shows in the build ----
    barrier0 = (lambda: dist.barrier()) if torchrun else (lambda: None)
    barrier0()
    t_att0 = time.perf_counter()
    top.synth_packets(SEED, args.hosts, 0, 10**9, window0)
    t_att1 = time.perf_counter()
    attach_phase_s = t_att1 - t_att0
    # the cold build's window starts here.  Library mode: Shadow's first packet calls the getters,
    # which derive the table geometry themselves (part of the first build); torchrun mode needs the
    # column count for its shards first.
    V, E = top.num_vertices, top.num_edges
    attached = None if library else top.attached_vertices()
    A = None if library else len(attached)

    kernel_ms, replay_ms = [], []
    if library:
        gmin_box = [None]

        def step():
            top.rebuild()  # rows on every device, exchange, table installed (shdtopo_rebuild)
            st_ = top.stats()
            kernel_ms.append(st_["sssp_kernel_ms"])
            replay_ms.append(st_["replay_ms"])
            gmin_box[0] = top.getMinimumLatency()

        def current_gmin():
            return gmin_box[0]
    else:
        table = sharding.ShardedTable(A, rank, world, dev)
        builder = sharding.hip_builder(top)

        def step():
            table.build(builder)
            st_ = top.stats()
            kernel_ms.append(st_["sssp_kernel_ms"])
            replay_ms.append(st_["replay_ms"])
            table.exchange()
            lr, hops = table.table()
            top.bind_table_ref(lr, hops, float(table.gmin.item()),
                               stream=torch.cuda.current_stream().cuda_stream)

        def current_gmin():
            return float(table.gmin.item())

    def barrier():
        if torchrun:
            dist.barrier()
        for d in range(ngpu if library else 1):
            torch.cuda.synchronize(d if library else local)

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        if torchrun:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---- cold build: the first table of the loaded topology, right after the attach phase.  In
    # library mode it is what Shadow's first packet triggers: topology_getLatency of two hosts
    # (shd-worker.c:360) builds the whole table and answers from its first copied row ----
    first_lat = None
    if library:
        first_lat = top.latency_ip(sa.ip_to_network("11.0.0.1"), sa.ip_to_network("11.0.0.2"))
        assert first_lat > 0, "the first getter failed"
    else:
        step()
    barrier()
    t1 = time.perf_counter()
    cold_s = max_over_ranks(t1 - t_att1)
    attach_to_table_s = max_over_ranks(t1 - t_att0)
    st_cold = top.stats()
    if attached is None:
        attached = top.attached_vertices()
        A = len(attached)
    # the packet window (same seed chain: every host re-attaches to the same vertex, the table
    # stays valid), then the timed steps
    tw0 = time.time()
    pk = top.synth_packets(SEED, args.hosts, args.packets, 10**9, window0)
    log(rank, "workload ready (window of %d packets in %.1fs): V=%d E=%d A=%d, %d GPU(s), mode %s"
        % (args.packets, time.time() - tw0, V, E, A, ngpu, args.mode))
    kernel_ms.clear()
    replay_ms.clear()
    for _ in range(args.warmup):
        step()
    kernel_ms.clear()
    replay_ms.clear()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    t_step = max_over_ranks(time.perf_counter() - t0) / args.steps
    st = top.stats()
    gmin = current_gmin()
    jump = int(gmin) * 1_000_000 if gmin >= 1.0 else window0   # shd-master.c:113-124
    gteps = A * E / t_step / 1e9

    # ---- packet routes: the window split over the GPUs, inputs resident in HBM ----
    nslice = ngpu if library else 1
    sl = []
    for s in range(nslice):
        p0, p1 = sharding.packet_range(args.packets, s if library else rank,
                                       ngpu if library else world)
        d = torch.device("cuda", s if library else local)
        cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(d)
        n = p1 - p0
        sl.append(dict(n=n, src=cu(pk["src_col"][p0:p1]), dst=cu(pk["dst_col"][p0:p1]),
                       pay=cu(pk["payload"][p0:p1].view(np.int32)),
                       sin=cu(pk["state_in"][p0:p1].view(np.int32)),
                       now=cu(pk["now"][p0:p1].view(np.int64)),
                       t=torch.empty(n, dtype=torch.int64, device=d),
                       s=torch.empty(n, dtype=torch.int32, device=d),
                       dl=torch.empty(n, dtype=torch.uint8, device=d)))

    def route_once():
        for s, x in enumerate(sl):
            if library:
                top.route_batch_device_slot(s, x["src"], x["dst"], x["pay"], x["sin"], x["now"],
                                            jump, 1, x["t"], x["s"], x["dl"])
            else:
                top.route_batch_device(x["src"], x["dst"], x["pay"], x["sin"], x["now"], jump, 1,
                                       x["t"], x["s"], x["dl"],
                                       stream=torch.cuda.current_stream().cuda_stream)
    route_ms = []
    for i in range(2 + args.route_steps):
        if i == 2:
            barrier()
            tr0 = time.perf_counter()
        route_once()
        if i >= 2:
            route_ms.append(top.stats()["route_kernel_ms"])  # slot 0's launch
    barrier()
    t_window = max_over_ranks(time.perf_counter() - tr0) / args.route_steps
    routes_per_s = args.packets / t_window

    getters = None
    if library and rank == 0 and args.getter_queries > 0:
        log(rank, "getters block: %d queries..." % args.getter_queries)
        getters = getters_block(top, pk, args.getter_queries, cpu_share(),
                                cpu=ngpu == 1 and not args.no_cpu_baseline)

    if rank == 0:
        srch = source_hash()
        rows = A if library else (table.r1 - table.r0)
        K = int(st["batch"])
        tie_dense = bool(st["tie_dense"])
        k_ms = float(np.mean(kernel_ms))
        r_ms = float(np.mean(replay_ms))
        wl = "C4%s" % ("int" if args.integer else "")
        key = "%s-%d-%d-%d-rows%d-gpus%d-%s" % (wl, V, E, A, rows, ngpu, srch)
        if tie_dense:
            # C4-int: every row through the exact heap replay, the batch kernel does not run
            pm = load_pmc(os.path.join(ROOT, "profiles", "%s_replay_pmc.json" % args.pmc_tag),
                          key + "-heap_replay_kernel")
            roofline = hbm_roofline(
                "heap_replay_kernel", r_ms, pm, 0, rows,
                "latency-bound: one wavefront walks igraph's sequential two-way heap per row; no "
                "algorithmic byte model applies (per row: %d pops, %d pushes, %d modifies)" % (
                    st["replay_pops"] // max(1, rows), st["replay_pushes"] // max(1, rows),
                    st["replay_modifies"] // max(1, rows)))
            roofline["model"] = None
            if pm and pm.get("lines_per_pop"):
                roofline["lines_per_pop"] = pm["lines_per_pop"]
        else:
            pm = load_pmc(os.path.join(ROOT, "profiles", "%s_sssp_pmc.json" % args.pmc_tag),
                          key + "-sssp_batch_kernel")
            roofline = hbm_roofline(
                "sssp_batch_kernel<%d>" % K, k_ms, pm, 24 * E + 20 * V, rows,
                "SURVEY.md 8(d): a full Dijkstra scan per source (24E + 20V bytes); the pruned "
                "batch kernel touches a fraction of it, so this equivalent rate exceeds the HBM "
                "peak and is not a bandwidth -- achieved / frac above are the measured bytes")
        roofline["pmc_key"] = key
        if not tie_dense:
            roofline["model_batched"] = batched_model(st, rows * A, k_ms, roofline.get("traffic"))
        sssp = dict(kernel=roofline["kernel"], batch=K, lds_hubs=int(st["lds_hubs"]),
                    sweeps=int(st["far_splits"]), slots=st["slots"],
                    workspace_gb=round(st["workspace_bytes"] / 1e9, 2),
                    batch_fill=int(st["batch_fill"]),
                    phase_ms_per_source=[round(x / max(1, rows), 3) for x in st["phase_ms"]],
                    parent_phase_ms_per_source=[round(x / max(1, rows), 3)
                                                for x in st["parent_phase_ms"]],
                    touched_lines_per_build=int(st["touched_lines"]),
                    walk_steps_per_source=round(st["walk_steps"] / max(1, rows)),
                    walk_kinds_per_source=dict(zip(("tree", "tail_improver", "hub_improver",
                                                    "row_scan"),
                                                   [round(x / max(1, rows)) for x in st["walk_kinds"]])),
                    tie_dense=tie_dense)
        # cold build: the first table of the loaded topology, split into its parts
        cs = st_cold
        # the first build's wait for the attach-time preparation: the library's lock wait (build
        # and geometry), at most the part of the preparation the attach phase did not hide
        cold_wait_ms = (cs["build_wait_ms"] if library else
                        max(0.0, min(cs["attach_prep_ms"], cs["first_attach_to_table_ms"] -
                                     attach_phase_s * 1e3 - cs["build_wall_ms"])))
        host_ms = cs["csr_host_ms"] + cs["csr_copy_ms"] + cs["order_ms"] + cs["replay_prep_ms"]
        cold = dict(
            ms=round(cold_s * 1e3, 2), gteps=round(A * E / cold_s / 1e9, 3),
            graph_prep_ms=round(cs["csr_ms"], 2), graph_prep_host_ms=round(cs["csr_host_ms"], 2),
            graph_prep_copy_ms=round(cs["csr_copy_ms"], 2), h0_rounds=int(cs["csr_h0_rounds"]),
            graph_prep_steps_ms=dict(zip(("upload", "relabel", "rows", "h0_distances", "h0_tree",
                                          "kappa_copy", "copies_out"),
                                         [round(x, 2) for x in cs["csr_step_ms"][:7]])),
            workspace_ms=round(cs["workspace_ms"], 2),
            target_prep_ms=round(cs["target_prep_ms"], 2),
            target_kappa_iters=int(cs["target_kappa_iters"]),
            order_ms=round(cs["order_ms"], 2), kernel_ms=round(cs["sssp_kernel_ms"], 2),
            replay_prep_ms=round(cs["replay_prep_ms"], 2), replay_ms=round(cs["replay_ms"], 2),
            exchange_ms=round(cs["exchange_ms"], 2),
            build_wall_ms=round(cs["build_wall_ms"], 2),
            build_steps_ms=dict(zip(("device_init", "geometry_table_alloc", "prep_to_launch",
                                     "sssp_kernel", "replay_rest", "stats"),
                                    [round(x, 2) for x in cs["build_step_ms"][:6]])),
            module_load_ms=round(cs["module_load_ms"], 2),
            build_wait_ms=round(cold_wait_ms, 2),
            attach_prep_ms=round(cs["attach_prep_ms"], 2),
            prep_trigger={0: "none", 1: "first attach", 2: "topology_new"}.get(
                int(cs["prep_trigger"]), "?"),
            attach_prep_steps_ms=dict(zip(("device_init", "graph_prep", "edge_scan", "workspace"),
                                          [round(x, 2) for x in cs["attach_prep_step_ms"]])),
            attach_phase_ms=round(attach_phase_s * 1e3, 2),
            first_attach_to_table_ms=round(attach_to_table_s * 1e3, 2),
            trigger="first topology_getLatency (library mode)" if library else "shdtopo_build_rows",
            first_getter_ms=round(attach_to_table_s * 1e3, 2) if library else None,
            getter_beyond_build_ms=round(cold_s * 1e3 - cs["build_wall_ms"] - cold_wait_ms, 2)
            if library else None,
            library_first_attach_to_table_ms=round(cs["first_attach_to_table_ms"], 2),
            serialised_ms=round(cs["attach_prep_ms"] + cold_s * 1e3 - cold_wait_ms, 2),
            tie_probe=dict(rows=int(cs["tie_probe_rows"]), flagged=int(cs["tie_probe_flagged"]),
                           ms=round(cs["tie_probe_ms"], 2)),
            host_ms=round(host_ms, 2), host_frac=round(host_ms / (cold_s * 1e3), 4),
            host_preparations=int(cs["csr_host_runs"]),
            note="ms = the first getter (library mode: topology_getLatency of hosts 0 -> 1, which "
                 "builds the whole table and answers from one copied row; first_getter_ms = first "
                 "attach -> that answer; getter_beyond_build_ms = its time outside the build and "
                 "the lock wait), made right after the attach phase (attach_phase_ms: "
                 "%d hosts, wall clock); device init, graph preparation and the workspace run "
                 "in a background thread (attach_prep_ms) started by prep_trigger (topology_new "
                 "after the parse, else the first attach), and the build waits build_wait_ms "
                 "for the rest of it; "
                 "first_attach_to_table_ms = first attach -> first table installed (wall clock); "
                 "serialised_ms = the preparation and the build one after the other (nothing "
                 "overlapped); host_ms = host work of the cold build (graph preparation copies + "
                 "host compute, source ordering, replay CSR); the rest runs on the GPU(s)" %
                 args.hosts)
        route_roof = None
        if sl:
            rkey = "C5-%d-%d-%d-%s-packet_route_kernel" % (sl[0]["n"], A, ngpu, srch)
            rpm = load_pmc(os.path.join(ROOT, "profiles", "%s_route_pmc.json" % args.pmc_tag), rkey)
            rk = float(np.mean(route_ms))
            route_roof = hbm_roofline("packet_route_kernel", rk, rpm, 53, sl[0]["n"],
                                      "SURVEY.md 8(d): 53 B per packet (24 B in, one 16-B record "
                                      "gather, 13 B out)")
            route_roof["pmc_key"] = rkey
            if rpm:
                route_roof["traffic_over_model"] = round(rpm["hbm_bytes_per_launch"] /
                                                         (53 * sl[0]["n"]), 3)
        cpu = None
        if ngpu == 1 and not args.no_cpu_baseline:
            nt = cpu_share()
            log(rank, "cpu baseline: %d sources on 1 thread, %d on %d threads..." % (
                args.cpu_sample, args.cpu_sample_mt, nt))
            cpu = cpu_baseline(top, attached, args.cpu_sample, args.cpu_sample_mt, nt)
            # C5: the whole window over the pre-built table (the table gather is done first,
            # outside the timed region), 1 thread and every thread of the job's share
            a_, lat_t, rel_t_, _ = top.table()
            rl = lat_t[pk["src_col"], pk["dst_col"]]
            rr = rel_t_[pk["src_col"], pk["dst_col"]]
            del lat_t, rel_t_
            cpu["packet_routes_per_s"] = cpu_route_baseline(
                rl, rr, pk["payload"], pk["state_in"], pk["now"], jump, 1)
            cpu["packet_routes_per_s_all_cores"] = cpu_route_baseline(
                rl, rr, pk["payload"], pk["state_in"], pk["now"], jump, nt)
            cpu["packet_route_sample"] = "the whole %d-packet window" % len(rl)
            cpu["host_nproc"] = os.cpu_count()
            cpu["job_cpu_share"] = nt
        complete = None
        if library and not args.no_complete:
            # configs 2 / 3 on the job's GPUs (option devices = N; "--opt devices=N" rehearses the
            # N-engine path on one GPU, the engines then sharing it)
            ndev = int(float(dict(kv.split("=") for kv in args.opt).get("devices", ngpu)))
            complete = complete_table_lines(nthreads=cpu_share(), devices=ndev, cpu=ngpu == 1)
        directed = None
        if library and ngpu == 1 and not args.no_directed and not args.integer:
            # after the main topology's buffers are gone (its workspace holds ~110 GB)
            top.free()
            torch.cuda.empty_cache()
            log(rank, "C4-dir line...")
            directed = directed_line(args.hosts)
        out = {
            "metric": "routing-table build GTEPS + packet-routes/sec at 1/2/4/8 MI355X "
                      "(%HBM roofline)",
            "value": round(gteps, 3),
            "unit": "GTEPS",
            "n_gpus": ngpu,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": "%s synthetic power-law topology (1M vertices / 10M undirected edges, "
                            "seed 20261015): full attached-vertex table, all %d sources x %d "
                            "targets; C5: %d hosts, %d packets per window" %
                            ("C4-int" if args.integer else "C4", A, A, args.hosts, args.packets),
                "vertices": V, "edges": E, "sources": A, "targets": A,
                "packets_per_window": args.packets, "hosts": args.hosts,
                "parallelism": ("%d GPU(s) driven by one process (library option devices): rows "
                                "sharded, RCCL all-gather + all-reduce(min)" % ngpu) if library
                               else ("%d processes: rows sharded, torch.distributed RCCL "
                                     "all-gather + all-reduce(min)" % world),
            },
            "cold_build": cold,
            "packet_routes_per_s": round(routes_per_s, 1),
            "ms_per_window": round(t_window * 1e3, 4),
            "roofline": roofline,
            "route_roofline": route_roof,
            "getters": getters,
            "sssp": sssp,
            "cpu_baseline": cpu,
            "runahead_min_latency_ms": gmin,
            "graphml": graphml,
            "complete_tables": complete,
            "directed": directed,
            "ambiguous_pairs": st["ambiguous_pairs"],
            "exchange": dict(kind={0: "none", 1: "rccl", 2: "push"}.get(
                int(st["exchange_kind"]), "?") if library else "torch.distributed",
                             ms=round(st["exchange_ms"], 2),
                             ms_exposed=round(st["exchange_exposed_ms"], 2) if library else None,
                             devices=int(st["devices"]) if library else world,
                             device_kernel_ms=[round(x, 3) for x in
                                               st["device_kernel_ms"][:min(8, int(st["devices"]))]]
                             if library and st["devices"] > 1 else None,
                             device_build_ms=[round(x, 3) for x in
                                              st["device_build_ms"][:min(8, int(st["devices"]))]]
                             if library and st["devices"] > 1 else None,
                             device_rows=st["device_rows"][:min(8, int(st["devices"]))]
                             if library and st["devices"] > 1 else None,
                             bytes_per_device=int(st["exchange_bytes"]) if library else
                             int((world - 1) * (table.r1 - table.r0) * (A * 18 + 8)),
                             gb_per_s_per_device=round(int(st["exchange_bytes"]) / 1e6 /
                                                       max(1e-9, st["exchange_ms"]), 2)
                             if library and st["exchange_ms"] > 0 else None),
            # rows whose target chains cross a d-tied parent, recomputed in igraph's heap pop order
            # by heap_replay_kernel (its time is inside ms_per_step and stated separately here)
            "replay": dict(rows=st["replay_rows"], ms=round(r_ms, 3),
                           pops=st["replay_pops"], pushes=st["replay_pushes"],
                           modifies=st["replay_modifies"], slots=st["replay_slots"],
                           int_keys=st["replay_int_keys"]),
            "slots": st["slots"],
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
