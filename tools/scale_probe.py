"""Probe: strong-scaling granularity of the C4 table build.  Times the first shard (rows
[0, ceil(A/N))) on one GPU for N = 1, 2, 4, 8 -- what each rank of an N-GPU job runs -- with the
batch size K = 8 and K = 4.  usage: python tools/scale_probe.py [integer]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

integer = len(sys.argv) > 1 and sys.argv[1] == "integer"
t0 = time.time()
top = sa.Topology.synthetic(seed=20261015, integer_latency=integer)
top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)
A = len(top.attached_vertices())
print("gen %.1fs A=%d" % (time.time() - t0, A), flush=True)
lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
for K, fill in ((8, 8), (8, 0)):
    top.set_option("batch", K)
    top.set_option("batch_fill", fill)
    top.build_rows_into(0, 64, lr[:64], hp[:64])  # workspace + warm
    for n in (1, 2, 4, 8):
        rows = -(-A // n)
        torch.cuda.synchronize()
        t0 = time.time()
        top.build_rows_into(0, rows, lr[:rows], hp[:rows])
        torch.cuda.synchronize()
        st = top.stats()
        print("K=%d fill=%d N=%d rows=%d wall %.1f ms kernel %.1f ms (x N = %.1f ms of one-GPU work)" % (
            K, st["batch_fill"], n, rows, (time.time() - t0) * 1e3, st["sssp_kernel_ms"], st["sssp_kernel_ms"] * n),
            flush=True)
