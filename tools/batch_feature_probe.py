"""Probe: which host feature predicts a batch's cost in the cold build's batch order (GPU box).

Builds the C4 table once with the default batches (8 sources, the grouping order) under
SHD_BATCH_TRACE, so every traced batch is one launch batch with its duration; relates the
durations to per-batch aggregates (mean / max) of source features from the h0 tree the engine
prepared (shdtopo_export_csr): depth, log of the top-branch size, log of the own subtree size, pi.
Prints correlations and the tail a longest-predicted-first order would leave.

usage: python tools/batch_feature_probe.py OUT
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

out = sys.argv[1]
trace = out + ".trace"
if os.path.exists(trace):
    os.unlink(trace)
os.environ["SHD_BATCH_TRACE"] = trace
top = sa.Topology.synthetic(seed=20261015)
top.synth_packets(20261015, 100_000, 0, 10**9, 10**7)
A = len(top.attached_vertices())
rows = A
lr = torch.empty((rows, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((rows, A), dtype=torch.int16, device="cuda")
top.set_option("balance", 0)
top.build_rows_into(0, rows, lr, hp)
torch.cuda.synchronize()
csr = top.export_csr()
raw = np.fromfile(trace, dtype=np.int64)
nb, kf, slots, nr = (int(x) for x in raw[:4])
W = 12  # kBTraceWords
bt = raw[4:4 + W * nb].reshape(nb, W).astype(np.float64)
sp = raw[4 + W * nb:4 + W * nb + 2 * nr].reshape(nr, 2)
src = sp[:, 0].astype(np.int64)
dur = (bt[:, 1] - bt[:, 0]) * 1e-5  # ms (100 MHz wall clock)
par = csr["tree_parent"].astype(np.int64)
V = len(par)
pot = csr["pot"]
h0 = int(np.argmin(pot))
order = np.argsort(pot, kind="stable")
depth = np.zeros(V, np.int64)
top_branch = np.arange(V)
for v in order:
    p = par[v]
    if p < V and v != h0:
        depth[v] = depth[p] + 1
        top_branch[v] = v if p == h0 else top_branch[p]
size = np.ones(V, np.int64)
for v in order[::-1]:
    p = par[v]
    if p < V and v != h0:
        size[p] += size[v]
feat = {"depth": depth[src], "log_branch": np.log1p(size[top_branch[src]]),
        "log_subtree": np.log1p(size[src]), "pi": pot[src]}
print("batches %d (fill %d) slots %d; dur ms p50 %.2f p90 %.2f max %.2f" % (
    nb, kf, slots, np.median(dur), np.percentile(dur, 90), dur.max()))
for name, f in feat.items():
    fb = f[:nb * kf].reshape(nb, kf)
    for agg, x in (("mean", fb.mean(1)), ("max", fb.max(1))):
        print("corr(dur, %s %s) %.3f" % (agg, name, np.corrcoef(dur, x)[0, 1]))
np.savez(out, dur=dur, src=src, **feat)
