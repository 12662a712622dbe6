"""Quick GPU probe: C4 synthetic graph, time the SSSP rows kernel on a row range."""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=256)
ap.add_argument("--delta", type=float, default=0)
ap.add_argument("--slots", type=int, default=0)
ap.add_argument("--opt", action="append", default=[], help="key=value library option")
ap.add_argument("--routers", type=int, default=990_000)
ap.add_argument("--poi", type=int, default=10_000)
ap.add_argument("--edges", type=int, default=10_000_000)
ap.add_argument("--hosts", type=int, default=100_000)
ap.add_argument("--reps", type=int, default=2)
args = ap.parse_args()

t = time.time()
top = sa.Topology.synthetic(n_routers=args.routers, n_poi=args.poi, n_edges=args.edges)
print("graph %.1fs V=%d E=%d" % (time.time() - t, top.num_vertices, top.num_edges), flush=True)
if args.delta:
    top.set_option("delta", args.delta)
if args.slots:
    top.set_option("slots", args.slots)
for kv in args.opt:
    k, v = kv.split("=")
    top.set_option(k, float(v))
t = time.time()
pk = top.synth_packets(20261015, args.hosts, 1000, 10**9, 10**7)
A = len(top.attached_vertices())
print("attach %.1fs A=%d" % (time.time() - t, A), flush=True)
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
    E = top.num_edges
    print("rep %d rows=%d wall %.3fs kernel %.3fms  GTEPS %.2f  relax/src %.3g  amb %d err %d long %d"
          % (rep, rows, dt, st["sssp_kernel_ms"], rows * E / (st["sssp_kernel_ms"] / 1e3) / 1e9,
             st["relaxations"] / rows, st["ambiguous_pairs"], st["errors"], st["long_paths"]),
          flush=True)
    print("   batches %d (measured layout %d), fill %d, order %.2f ms" % (
        st["batches"], st["batch_layout_measured"], st["batch_fill"], st["order_ms"]), flush=True)
    ph = st["phase_ms"]
    print("   per-source ms: init %.2f sssp %.2f parents %.2f targets %.2f | near-it/src %.0f "
          "splits/src %.0f slots %d" % tuple([x / rows for x in ph] +
                                            [st["near_iterations"] / rows,
                                             st["far_splits"] / rows, st["slots"]]), flush=True)
    print("   parent phases ms/src: walks %.3f scans %.3f recount %.3f next %.3f" %
          tuple(x / rows for x in st["parent_phase_ms"]), flush=True)
    print("   walk steps/src %.0f, walk kinds %s" % (st["walk_steps"] / rows, list(st["walk_kinds"])),
          flush=True)
    print("   target prep %.2f ms (%d kappa iterations)" % (st["target_prep_ms"],
                                                         st["target_kappa_iters"]), flush=True)
    print("   split ms/src %.2f  far-scan sources %d" % (st["split_ms"] / rows,
                                                      st["far_scan_sources"]), flush=True)
    if any(st["batch_wave_ms"]):
        w = st["batch_wave_ms"]
        print("   wave ms/src (SHD_BATCH_TIME): tail chunk %.2f A %.2f B %.2f | hub chunk %.2f A %.2f "
              "B %.2f | phase-B rounds/src %.0f pairs/src %.0f (%.2f per round)" % tuple(
                  [x / rows for x in w] + [st["batch_rounds"] / rows, st["batch_edges_b"] / rows,
                                           st["batch_edges_b"] / max(1, st["batch_rounds"])]),
              flush=True)
    if any(st.get("sweep_events", [0])):
        sw = st["sweep_events"]
        print("   phase B (SHD_BATCH_TIME) per source: rounds with a tail target %.0f, tail-target "
              "pairs %.0f, hub-target pairs %.0f" % tuple(x / rows for x in sw[:3]), flush=True)
    if any(st.get("write_lines", [0])):
        names = ("relax_min", "relax_tie", "relax_hint", "relax_pend", "relax_touch", "relax_mask",
                 "mask_st", "pend_st", "reset", "touch_clr", "prec", "pscr", "out", "hub", "queue",
                 "other")
        wl = st["write_lines"]
        print("   write lines per source (SHD_BATCH_WRCOUNT): total %.0f %s" % (
            sum(wl) / rows, {k: round(v / rows) for k, v in zip(names, wl)}), flush=True)
        rl = st["read_lines"]
        print("   read lines per source (SHD_BATCH_WRCOUNT): total %.0f %s" % (
            sum(rl) / rows, {k: round(v / rows) for k, v in zip(
                ("pre", "phase_a", "chunk", "sweep", "walk", "epi", "reset", "other"), rl)}),
            flush=True)
    print("   per-source events:", {k: "%.3g" % (v / rows) for k, v in st["events"].items()},
          flush=True)
x = lr[..., 0].cpu().numpy()
print("lat min %.4f max %.4f mean %.3f" % (x.min(), x.max(), x.mean()))
h = hp.cpu().numpy()
print("hops max %d mean %.2f" % (h.max(), h.mean()))
