"""Probe: a directed topology through the batched SSSP (GPU box).

C4-dir: the C4 synthetic generator with directed = 1 -- every non-loop edge of the 1M-vertex /
10M-edge power-law graph becomes two arcs, the reverse one with its own latency and loss draw
(E = 19.99 M arcs).  Times the table rows [0, ROWS) through the batch kernel (out-rows relaxed,
parents from the in-rows) against the exact heap replay alone (replay_all, a sample of rows,
extrapolated per row), and checks the batch rows' latencies against scipy's directed Dijkstra on
a few sources (same left-to-right f64 sums: bit-exact).

usage: python tools/directed_probe.py [--rows 10000] [--reps 2] [--replay-rows 256] [--check 4]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--replay-rows", type=int, default=256)
ap.add_argument("--check", type=int, default=4)
ap.add_argument("--routers", type=int, default=990_000)
ap.add_argument("--poi", type=int, default=10_000)
ap.add_argument("--edges", type=int, default=10_000_000)
ap.add_argument("--integer", type=int, default=0)
ap.add_argument("--opt", action="append", default=[], help="key=value library option")
args = ap.parse_args()


def make():
    t = time.time()
    top = sa.Topology.synthetic(n_routers=args.routers, n_poi=args.poi, n_edges=args.edges,
                                integer_latency=bool(args.integer), directed=True)
    assert top.is_directed
    for kv in args.opt:
        k, v = kv.split("=")
        top.set_option(k, float(v))
    top.synth_packets(20261015, 100_000, 0, 10**9, 10**7)  # attaches the hosts
    print("graph + attach %.1fs V=%d E=%d A=%d" % (time.time() - t, top.num_vertices,
                                                    top.num_edges, len(top.attached_vertices())),
          flush=True)
    return top


top = make()
A = len(top.attached_vertices())
E = top.num_edges
rows = min(args.rows, A)
lr = torch.empty((rows, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((rows, A), dtype=torch.int16, device="cuda")
for rep in range(args.reps):
    torch.cuda.synchronize()
    t = time.time()
    top.build_rows_into(0, rows, lr, hp)
    torch.cuda.synchronize()
    dt = time.time() - t
    st = top.stats()
    print("batch rep %d rows=%d wall %.1f ms kernel %.2f ms (%.1f GTEPS)  replay rows %d (%.1f ms)  "
          "ambiguous %d errors %d csr %.1f ms target prep %.1f ms" % (
              rep, rows, dt * 1e3, st["sssp_kernel_ms"],
              rows * E / (st["sssp_kernel_ms"] / 1e3) / 1e9, st["replay_rows"], st["replay_ms"],
              st["ambiguous_pairs"], st["errors"], st["csr_ms"], st["target_prep_ms"]), flush=True)

# latencies against scipy's directed Dijkstra (the same f64 sums from the source)
if args.check > 0:
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    eu, ev, elat = np.asarray(eu), np.asarray(ev), np.asarray(elat)
    nl = eu != ev
    W = sp.csr_matrix((elat[nl], (eu[nl], ev[nl])), shape=(V, V))
    assert W.nnz == int(nl.sum())
    verts = np.asarray(top.attached_vertices(), np.int64)
    lat = lr[:, :, 0].cpu().numpy()
    # the table's rows are the attached vertices in column order
    srcs = list(range(min(args.check, rows)))
    d = dijkstra(W, directed=True, indices=verts[srcs])
    bad = 0
    for i, r in enumerate(srcs):
        ref = d[i][verts]
        ref[r] = lat[r, r]  # the self pair is the self loop (shd-topology.c:561-671)
        bad += int(np.sum(ref.view(np.uint64) != lat[r].view(np.uint64)))
    print("scipy directed check: %d rows x %d targets, %d latencies differ" % (len(srcs), A, bad),
          flush=True)
    del W

# the replay alone on a sample of rows (the path directed topologies took before)
if args.replay_rows > 0:
    n = min(args.replay_rows, rows)
    top.set_option("replay_all", 1)
    torch.cuda.synchronize()
    t = time.time()
    top.build_rows_into(0, n, lr[:n], hp[:n])
    torch.cuda.synchronize()
    st = top.stats()
    ms = st["replay_ms"]
    # n <= slots rows run as one round of wavefronts, so the full table takes about
    # ceil(rows / slots) such rounds
    slots = max(1, st["replay_slots"])
    print("replay_all rows=%d wall %.1f ms replay %.1f ms (one round of %d slots) -> full %d rows "
          "~ %.1f s" % (n, (time.time() - t) * 1e3, ms, slots, rows,
                        -(-rows // slots) * ms / 1e3), flush=True)
