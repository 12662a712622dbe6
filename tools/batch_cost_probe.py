"""Probe: what predicts a source's cost in sssp_batch_kernel (GPU box, C4 synthetic graph).

Runs ROWS sources once with batches of one source (batch_fill 1) under SHD_BATCH_TRACE, so every
traced batch is one source's relaxations / expansions / duration, then relates them to features
of the source in the h0 shortest-path tree the engine prepared (shdtopo_export_csr): pi, tree
depth, the size of the source's own subtree and of its top branch (the subtree below h0 that
holds it), and its degree.  Prints correlations and writes OUT.npz for offline study.

usage: python tools/batch_cost_probe.py OUT [ROWS]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import shadow_amd as sa  # noqa: E402

out = sys.argv[1]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1250
trace = out + ".trace"
if os.path.exists(trace):
    os.unlink(trace)
os.environ["SHD_BATCH_TRACE"] = trace
top = sa.Topology.synthetic(seed=20261015)
top.synth_packets(20261015, 100_000, 0, 10**9, 10**7)
A = len(top.attached_vertices())
lr = torch.empty((rows, A, 2), dtype=torch.float64, device="cuda")
hp = torch.empty((rows, A), dtype=torch.int16, device="cuda")
top.set_option("batch_fill", 1)
top.build_rows_into(0, rows, lr, hp)
torch.cuda.synchronize()
csr = top.export_csr()
raw = np.fromfile(trace, dtype=np.int64)
nb, kf, slots, nr = (int(x) for x in raw[:4])
W = 12  # kBTraceWords
bt = raw[4:4 + W * nb].reshape(nb, W).astype(np.float64)
sp = raw[4 + W * nb:4 + W * nb + 2 * nr].reshape(nr, 2)
src = sp[:, 0].astype(np.int64)
dur = (bt[:, 1] - bt[:, 0]) * 1e-5
rel, exp = bt[:, 6], bt[:, 5]

par = csr["tree_parent"].astype(np.int64)
V = len(par)
rowptr = csr["rowptr"].astype(np.int64)
deg = np.diff(rowptr)
pot = csr["pot"]
h0 = int(np.argmin(pot))
# depth and subtree sizes of the h0 tree (parents >= V: the root / unreachable)
order = np.argsort(pot, kind="stable")  # parents before children
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
feats = {
    "pi": pot[src], "depth": depth[src], "subtree": size[src],
    "branch": size[top_branch[src]], "deg": deg[src],
    "log_branch": np.log1p(size[top_branch[src]]),
}
print("rows %d batches %d (fill %d)  h0 %d" % (nr, nb, kf, h0))
print("per source: dur ms p50 %.2f p90 %.2f max %.2f | relax p50 %.3g max %.3g | exp p50 %.3g max %.3g" % (
    np.median(dur), np.percentile(dur, 90), dur.max(), np.median(rel), rel.max(), np.median(exp),
    exp.max()))
for name, y in (("relax", rel), ("exp", exp), ("dur", dur)):
    print("corr(%s, x): " % name + ", ".join("%s %.2f" % (k, np.corrcoef(y, v)[0, 1])
                                           for k, v in feats.items() if np.std(v) > 0))
np.savez(out, src=src, dur=dur, rel=rel, exp=exp, tree_parent=csr["tree_parent"], pot=pot,
         deg_all=deg.astype(np.int32), **feats)
