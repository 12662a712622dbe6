"""Probe: heap-replay cost on C4-int (integer latencies) for a row range, per row and per heap op.
usage: python tools/replay_probe.py ROWS [SLOTS] [all] [LANDMARK] [INT_KEYS]  (all: only the
replay_all mode; LANDMARK 0: no landmark skip; INT_KEYS 0: f64 heap keys)"""
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 256
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 0
t0 = time.time()
top = sa.Topology.synthetic(seed=20261015, integer_latency=True)
top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)
A = len(top.attached_vertices())
print("gen %.1fs A=%d" % (time.time() - t0, A), flush=True)
if slots:
    top.set_option("replay_slots", slots)
if len(sys.argv) > 4:
    top.set_option("replay_landmark", int(sys.argv[4]))
if len(sys.argv) > 5:
    top.set_option("replay_int_keys", int(sys.argv[5]))
lr = torch.empty((rows, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((rows, A), dtype=torch.int16, device="cuda")
modes = ("replay_all",) if len(sys.argv) > 3 and sys.argv[3] == "all" else ("batch+replay", "replay_all")
for mode in modes:
    top.set_option("replay_all", 1 if mode == "replay_all" else 0)
    t0 = time.time()
    top.build_rows_into(0, rows, lr, hp)
    torch.cuda.synchronize()
    st = top.stats()
    r = max(1, st["replay_rows"])
    print("%s: wall %.2fs sssp %.1f ms replay %.1f ms rows %d slots %d ambiguous %d | per row: "
          "pops %.0f pushes %.0f mods %.0f skips %.0f" % (
              mode, time.time() - t0, st["sssp_kernel_ms"], st["replay_ms"], st["replay_rows"],
              st["replay_slots"], st["ambiguous_pairs"], st["replay_pops"] / r,
              st["replay_pushes"] / r, st["replay_modifies"] / r, st["replay_skips"] / r), flush=True)
    if any(st["replay_lines"]):
        pops = max(1, st["replay_pops"])
        print("  64-B lines per pop: " + " ".join("%s %.1f" % (n, x / pops) for n, x in zip(
            ("sink_ld", "sink_st", "shift_ld", "shift_st", "relax_ld", "relax_st"),
            st["replay_lines"])) + " | total %.1f" % (sum(st["replay_lines"]) / pops), flush=True)
    if any(st["replay_phase_ms"]):
        pops = max(1, st["replay_pops"])
        print("  ns per pop (per wavefront): " + " ".join("%s %.0f" % (n, x * 1e6 / pops) for n, x in zip(
            ("sink", "loads", "heap_ops", "rest"), st["replay_phase_ms"])) +
            " | sink rounds %.2f, mean heap size %.0f" % (st["replay_sink_rounds"] / pops,
                                                         st["replay_heap_sum"] / pops), flush=True)
        print("  sink ns per pop: lds_walk %.0f hbm_rounds %.0f moves %.0f | prefetch hits %.3f" % (
            tuple(x * 1e6 / pops for x in st["replay_sink_ms"]) + (st["replay_pf_hits"] / pops,)),
            flush=True)
