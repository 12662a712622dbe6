"""Probe: every shard of an N-GPU C4 table build (rows [d*R, (d+1)*R), R = ceil(A/N)), timed one
after another on one GPU: the slowest shard bounds an N-GPU step's kernel time.
usage: python tools/scale_probe2.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

t0 = time.time()
top = sa.Topology.synthetic(seed=20261015)
top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)
A = len(top.attached_vertices())
print("gen %.1fs A=%d" % (time.time() - t0, A), flush=True)
lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
top.build_rows_into(0, A, lr, hp)  # workspace, target preparation
print("target prep %.1f ms" % top.stats()["target_prep_ms"], flush=True)
for n in (1, 2, 4, 8):
    R = -(-A // n)
    ks = []
    for d in range(n):
        r0, r1 = d * R, min(A, (d + 1) * R)
        top.build_rows_into(r0, r1, lr[: r1 - r0], hp[: r1 - r0])
        torch.cuda.synchronize()
        ks.append(top.stats()["sssp_kernel_ms"])
    print("N=%d rows/shard=%d kernel ms per shard: %s  max %.1f  (x N = %.1f)" % (
        n, R, " ".join("%.1f" % k for k in ks), max(ks), max(ks) * n), flush=True)
