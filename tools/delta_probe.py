"""Probe: batch-kernel time vs bucket width delta for shard sizes of N = 1, 4, 8 on C4.
usage: python tools/delta_probe.py [delta_ms ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

deltas = [float(x) for x in sys.argv[1:]] or [0.0, 20.0, 40.0, 80.0]
top = sa.Topology.synthetic(seed=20261015, integer_latency=False)
top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)
A = len(top.attached_vertices())
lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
top.build_rows_into(0, 64, lr[:64], hp[:64])
for d in deltas:
    top.set_option("delta", d)
    for n in (1, 4, 8):
        rows = -(-A // n)
        torch.cuda.synchronize()
        t0 = time.time()
        top.build_rows_into(0, rows, lr[:rows], hp[:rows])
        torch.cuda.synchronize()
        st = top.stats()
        print("delta=%s N=%d rows=%d kernel %.1f ms phases/source %s" % (
            d or "auto", n, rows, st["sssp_kernel_ms"],
            " ".join("%.2f" % (x / rows) for x in st["phase_ms"])), flush=True)
