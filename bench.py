#!/usr/bin/env python3
"""bench.py -- routing-table build GTEPS + packet-routes/s on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE.json configs 4 + 5; synthetic, generated in memory):
  * C4: power-law Internet topology, 990,000 routers + 10,000 poi, exactly 10,000,000 undirected
    edges (Chung-Lu, deduplicated, spanning path, poi uplinks + self loops), seed 20261015;
  * C5: 100,000 Tor-like hosts attached by type hint (94/5/1 % client/relay/server) through
    Shadow's seed chain; one scheduler window of 10,000,000 packets.
A step = one build of the whole attached-vertex routing table (all A ~ 10^4 sources x A targets:
near-far SSSP + parent/epilogue kernel per source, rows sharded over the ranks, RCCL all-gather of
the rows, all-reduce(MIN) of the runahead minimum, table installed in the library).
value = A * E / t_step / 1e9 (Graph500 SSSP convention, undirected E) = GTEPS, whole job.
Packet routes are timed separately over resident windows and reported as packet_routes_per_s.

Launch: python bench.py [--gpus 1 --steps K --warmup W]   or, for N > 1,
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import math
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

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SEED = 20261015


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


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
    timed on this host on bounded samples of sources: 1 thread (the reference's concurrency:
    Dijkstra runs under the global graphLock) and every thread of the job's CPU
    share (sources are independent); each extrapolated linearly by source count."""
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
               sample="%d of %d sources x %d targets (Dijkstra + per-target helper) on 1 thread, "
                      "%.1f s; extrapolated linearly to the full table: %.0f s" %
                      (len(srcs), A, A, t, t / len(srcs) * A),
               seconds_per_source=t / len(srcs), oracle_setup_s=t_setup)
    if n_sample_mt > 0 and nthreads_mt > 1:
        srcs = attached[n_sample:n_sample + n_sample_mt]
        t0 = time.time()
        g.source_rows(srcs, attached, nthreads=nthreads_mt)
        t = time.time() - t0
        out["all_cores"] = dict(
            value=len(srcs) * E / t / 1e9, unit="GTEPS", cores=nthreads_mt,
            sample="%d sources x %d targets on %d threads (the job's CPU share), %.1f s; "
                   "extrapolated to the full table: %.0f s" % (len(srcs), A, nthreads_mt, t,
                                                               t / len(srcs) * A),
            seconds_per_source=t / len(srcs))
    return out


def complete_table_lines(repeats=20):
    """BASELINE configs 2 (plab, 303 x 303) and 3 (full Internet, 183 x 183): the complete-graph
    pair table (_topology_lookupPath for every attached pair, shd-topology.c:835-873) on the
    GPU vs the oracle's restatement on one CPU thread.  One host per vertex via its unique
    geocode hint.  34 B per pair (roofline of pair_table_complete_kernel)."""
    import lzma
    import oracle
    out = {}
    for cfg, name in (("C2", "topology.plab"), ("C3", "topology")):
        path = os.path.join(ROOT, "tests", "golden", "resource", name + ".graphml.xml.xz")
        with lzma.open(path) as f:
            data = f.read()
        top = sa.Topology.from_buffer(data)
        g = oracle.OGraph.from_graphml(data)
        geos = list(g.vattrs["geocode"])
        st = 1
        for k, geo in enumerate(geos):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            top.attach_ip(sa.ip_to_network("11.%d.%d.%d" % (k >> 16, (k >> 8) & 255, k & 255)),
                          st, geocodeHint=geo)
        A = len(top.attached_vertices())
        lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
        hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
        rm = torch.empty((A,), dtype=torch.float64, device="cuda")
        ms = []
        for i in range(repeats + 2):
            top.build_rows_into(0, A, lr, hp, rm)
            if i >= 2:
                ms.append(top.stats()["sssp_kernel_ms"])
        k_ms = float(np.median(ms))
        a = np.asarray(sorted(set(top.attached_vertices().tolist())), np.int32)
        S, D = np.meshgrid(a, a, indexing="ij")
        t0 = time.perf_counter()
        g.complete_pairs(S.ravel(), D.ravel())
        t_cpu = time.perf_counter() - t0
        pairs = A * A
        out[cfg] = dict(topology=name, attached=A, pairs=pairs,
                        gpu_pairs_per_s=round(pairs / (k_ms / 1e3), 1), kernel_ms=round(k_ms, 4),
                        kernel="pair_table_complete_kernel + row_min_kernel",
                        roofline=dict(bound="hbm", bytes_per_unit=34, units_per_launch=pairs,
                                      achieved=round(pairs * 34 / (k_ms / 1e3) / 1e9, 2),
                                      peak=HBM_PEAK_GBS, unit="GB/s",
                                      frac=round(pairs * 34 / (k_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5)),
                        cpu_pairs_per_s=round(pairs / t_cpu, 1), cpu_cores=1,
                        note="launch-bound: %d pairs are a few microseconds of HBM time" % pairs)
    return out


def cpu_route_baseline(lat, rel, payload, state, now, jump):
    import oracle
    t0 = time.time()
    oracle.route_packets(lat, rel, payload, state, now, jump, 1)
    return len(lat) / (time.time() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--routers", type=int, default=990_000)
    ap.add_argument("--poi", type=int, default=10_000)
    ap.add_argument("--edges", type=int, default=10_000_000)
    ap.add_argument("--hosts", type=int, default=100_000)
    ap.add_argument("--packets", type=int, default=10_000_000)
    ap.add_argument("--route-steps", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=24,
                    help="sources timed on 1 CPU thread (about 1 s each)")
    ap.add_argument("--cpu-sample-mt", type=int, default=256,
                    help="sources timed on all threads of the job's CPU share")
    ap.add_argument("--no-graphml", action="store_true",
                    help="skip the GraphML write + topology_new load of the generated topology")
    ap.add_argument("--no-complete", action="store_true", help="skip the C2/C3 table lines")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--delta", type=float, default=0.0)
    ap.add_argument("--integer", action="store_true",
                    help="C4-int variant (integer latencies U{1..100}: heavy parent ties)")
    ap.add_argument("--batch", type=int, default=8,
                    help="sources per SSSP workgroup (1 = single-source sssp_rows_kernel)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "r02w_sssp_pmc.json"))
    ap.add_argument("--route-pmc-json", default=os.path.join(ROOT, "profiles", "r02w_route_pmc.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    # ---- workload (identical on every rank; generation and loading are outside the timed
    # region).  The generated C4 topology is written as GraphML once and loaded back through
    # topology_new (shd-topology.c:1237 -> _topology_loadGraph :95-123), as Shadow loads it;
    # the round trip must reproduce the generator's graph bit for bit. ----
    t0 = time.time()
    gen = sa.Topology.synthetic(seed=SEED, n_routers=args.routers, n_poi=args.poi,
                                n_edges=args.edges, integer_latency=args.integer)
    graphml = dict(generate_s=round(time.time() - t0, 2))
    top = gen
    if not args.no_graphml:
        import tempfile
        path = os.path.join(tempfile.gettempdir(), "shdtopo_c4_%s_%d.graphml.xml" % (
            "int" if args.integer else "real", os.getpid() if world == 1 else 0))
        if world > 1:
            path = path.replace("_0.graphml", "_%s.graphml" % os.environ.get("MASTER_PORT", "0"))
        try:
            if rank == 0:
                t1 = time.time()
                gen.write_graphml(path)
                graphml["write_s"] = round(time.time() - t1, 2)
                graphml["bytes"] = os.path.getsize(path)
            if world > 1:
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
            if world > 1:
                dist.barrier()
            if rank == 0 and os.path.exists(path):
                os.unlink(path)
    del gen
    top.set_option("device", local)
    top.set_option("batch", args.batch)
    if args.delta:
        top.set_option("delta", args.delta)
    window0 = 10_000_000  # Shadow's default 10 ms window until the runahead is known
    pk = top.synth_packets(SEED, args.hosts, args.packets, 10**9, window0)
    attached = top.attached_vertices()
    A, V, E = len(attached), top.num_vertices, top.num_edges
    log(rank, "workload ready in %.1fs: V=%d E=%d A=%d packets=%d" %
        (time.time() - t0, V, E, A, args.packets))

    table = sharding.ShardedTable(A, rank, world, dev)
    builder = sharding.hip_builder(top)
    kernel_ms = []
    replay_ms = []

    def step():
        table.build(builder)
        st_ = top.stats()
        kernel_ms.append(st_["sssp_kernel_ms"])
        replay_ms.append(st_["replay_ms"])
        table.exchange()
        lr, hops = table.table()
        top.bind_table(lr, hops, float(table.gmin.item()),
                       stream=torch.cuda.current_stream().cuda_stream)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    kernel_ms.clear()
    replay_ms.clear()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    t_step = float(elapsed.item()) / args.steps
    st = top.stats()
    gmin = float(table.gmin.item())
    jump = int(gmin) * 1_000_000 if gmin >= 1.0 else window0   # shd-master.c:113-124
    gteps = A * E / t_step / 1e9

    # ---- packet routes: this rank's slice of the window, inputs resident in HBM ----
    p0, p1 = sharding.packet_range(args.packets, rank, world)
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    d_src = cu(pk["src_col"][p0:p1])
    d_dst = cu(pk["dst_col"][p0:p1])
    d_pay = cu(pk["payload"][p0:p1].view(np.int32))
    d_sin = cu(pk["state_in"][p0:p1].view(np.int32))
    d_now = cu(pk["now"][p0:p1].view(np.int64))
    n = p1 - p0
    t_out = torch.empty(n, dtype=torch.int64, device=dev)
    s_out = torch.empty(n, dtype=torch.int32, device=dev)
    d_out = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    route_ms = []
    for i in range(2 + args.route_steps):
        if i == 2:
            barrier()
            tr0 = time.perf_counter()
        top.route_batch_device(d_src, d_dst, d_pay, d_sin, d_now, jump, 1, t_out, s_out, d_out,
                               stream=stream)
        if i >= 2:
            route_ms.append(top.stats()["route_kernel_ms"])
    barrier()
    rel_t = torch.tensor([time.perf_counter() - tr0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(rel_t, op=dist.ReduceOp.MAX)
    t_window = float(rel_t.item()) / args.route_steps
    routes_per_s = args.packets / t_window

    if rank == 0:
        # roofline of the dominant kernel (the SSSP launch), algorithmic bytes per source =
        # 2E (4 B col + 8 B weight) + V (4 B rowptr + 8 B dist read + 8 B dist write)
        rows = table.r1 - table.r0
        b_src = 24 * E + 20 * V
        k_s = float(np.mean(kernel_ms)) / 1e3
        achieved = rows * b_src / k_s / 1e9
        K = int(st["batch"])
        kname = "sssp_batch_kernel<%d>" % K if K > 1 else "sssp_rows_kernel"
        # the batch kernel's per-bucket sweeps read only the 64-B lines of vertices with a
        # pending bit (random 64-B requests, which FETCH_SIZE counts at their size): no streaming
        # correction (MI355X_MICROARCH.md: only wide coalesced 128-B reads are tallied at half)
        sweeps = int(st["far_splits"]) if K > 1 else 0
        sweep_bytes = 0
        traffic = None
        pmc_note = None
        pmc_requests = None
        if os.path.exists(args.pmc_json):
            try:
                pm = json.load(open(args.pmc_json))
                if not args.integer and pm.get("config_key") == "C4-%d-%d-%d-rows%d-%s" % (
                        V, E, A, rows, kname):
                    traffic = pm["hbm_bytes_per_launch"]
                    pmc_note = pm.get("source")
                    pmc_requests = pm.get("dram_requests_per_launch")
            except Exception:
                traffic = None
        roofline = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBS,
                        unit="GB/s", frac=round(achieved / HBM_PEAK_GBS, 5), traffic=traffic,
                        # measured HBM bytes (PMC) per launch / the launch time: what the memory
                        # system actually moved, beside the per-source model above
                        frac_measured=(round(traffic / k_s / 1e9 / HBM_PEAK_GBS, 5)
                                       if traffic else None),
                        dram_requests_per_source=(round(pmc_requests / rows)
                                                  if pmc_requests else None),
                        kernel=kname, kernel_ms=round(k_s * 1e3, 3),
                        units_per_launch=rows, bytes_per_unit=b_src, pmc=pmc_note)
        sssp = dict(kernel=kname, batch=K, lds_hubs=int(st["lds_hubs"]), sweeps=sweeps,
                    sweep_bytes=sweep_bytes, slots=st["slots"],
                    phase_ms_per_source=[round(x / max(1, rows), 3) for x in st["phase_ms"]],
                    # once per (graph, target set), in the warmup build: target bits and the
                    # target-aware kappa fixpoint in the relaxation copy (outside the timed steps,
                    # like the CSR upload and the h0 distances)
                    target_prep_ms=round(float(st["target_prep_ms"]), 2),
                    target_kappa_iters=int(st["target_kappa_iters"]))
        r_ms = float(np.mean(route_ms))
        route_roof = dict(bound="hbm", kernel="packet_route_kernel", kernel_ms=round(r_ms, 4),
                          achieved=round(n * 53 / (r_ms / 1e3) / 1e9, 1), peak=HBM_PEAK_GBS,
                          unit="GB/s", bytes_per_unit=53, units_per_launch=n)
        route_roof["frac"] = round(route_roof["achieved"] / HBM_PEAK_GBS, 4)
        route_roof["traffic"] = None
        if os.path.exists(args.route_pmc_json) and world == 1 and n == 10_000_000:
            try:
                rp = json.load(open(args.route_pmc_json))
                route_roof["traffic"] = rp["hbm_bytes_per_launch"]
                route_roof["frac_measured"] = round(
                    rp["hbm_bytes_per_launch"] / (r_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                route_roof["traffic_over_algorithmic"] = round(
                    rp["hbm_bytes_per_launch"] / (n * 53), 3)
            except Exception:
                pass
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            nt = cpu_share()
            log(rank, "cpu baseline: %d sources on 1 thread, %d on %d threads..." % (
                args.cpu_sample, args.cpu_sample_mt, nt))
            cpu = cpu_baseline(top, attached, args.cpu_sample, args.cpu_sample_mt, nt)
            nr = min(args.packets, 2_000_000)
            a_, lat_t, rel_t_, _ = top.table()
            cpu["packet_routes_per_s"] = cpu_route_baseline(
                lat_t[pk["src_col"][:nr], pk["dst_col"][:nr]],
                rel_t_[pk["src_col"][:nr], pk["dst_col"][:nr]], pk["payload"][:nr],
                pk["state_in"][:nr], pk["now"][:nr], jump)
            cpu["host_nproc"] = os.cpu_count()
            cpu["job_cpu_share"] = nt
        complete = None
        if world == 1 and not args.no_complete:
            complete = complete_table_lines()
        out = {
            "metric": "routing-table build GTEPS + packet-routes/sec at 1/2/4/8 MI355X "
                      "(%HBM roofline)",
            "value": round(gteps, 3),
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": "C4%s synthetic power-law topology (1M vertices / 10M undirected "
                            "edges, seed 20261015): full attached-vertex table, all %d sources x "
                            "%d targets; C5: %d hosts, %d packets per window" %
                            ("-int" if args.integer else "", A, A, args.hosts, args.packets),
                "vertices": V, "edges": E, "sources": A, "targets": A,
                "packets_per_window": args.packets, "hosts": args.hosts,
                "parallelism": "sources sharded /%d, RCCL all-gather + all-reduce(min)" % world,
            },
            "packet_routes_per_s": round(routes_per_s, 1),
            "ms_per_window": round(t_window * 1e3, 4),
            "roofline": roofline,
            "route_roofline": route_roof,
            "sssp": sssp,
            "cpu_baseline": cpu,
            "runahead_min_latency_ms": gmin,
            "graphml": graphml,
            "complete_tables": complete,
            "ambiguous_pairs": st["ambiguous_pairs"],
            # rows whose target chains cross a d-tied parent, recomputed in igraph's heap pop order
            # by heap_replay_kernel (its time is inside ms_per_step and stated separately here)
            "replay": dict(rows=st["replay_rows"], ms=round(float(np.mean(replay_ms)), 3),
                           pops=st["replay_pops"], pushes=st["replay_pushes"],
                           modifies=st["replay_modifies"], slots=st["replay_slots"]),
            "slots": st["slots"],
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
