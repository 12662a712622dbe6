"""The graph preparation on the GPU (topo_prep.hip) against a numpy/scipy
restatement: the relabel (degree order, tail grouped by primary hub), the CSR rows (ascending by
(neighbour, edge id)), pi = d(h0, .) (scipy's Dijkstra: left-to-right f64 sums, the same unique
fixpoint) and the h0 tree (argmin (d(u), u) over tight edges with d(u) < d(v)).

These arrays only shape performance -- every table is checked against the oracle elsewhere -- but
the relabel, rows and pi must be exactly what DESIGN.md describes for the kernels' bounds to hold.
"""
import time

import numpy as np
import pytest
import scipy.sparse as sp
from scipy.sparse.csgraph import dijkstra

import shadow_amd as sa

pytestmark = pytest.mark.gpu

GROUP_HUBS = 16565  # kGroupHubs (topo_core.cpp)


def restate(top):
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    nl = eu != ev
    a, b, w, e = eu[nl], ev[nl], elat[nl], np.nonzero(nl)[0]
    deg = np.bincount(a, minlength=V) + np.bincount(b, minlength=V)
    perm = np.argsort(-deg, kind="stable")
    H = min(GROUP_HUBS, V)
    if H < V:
        hubrank = np.full(V, np.iinfo(np.int32).max, np.int64)
        hubrank[perm[:H]] = np.arange(H)
        primary = np.full(V, np.iinfo(np.int32).max, np.int64)
        np.minimum.at(primary, a, hubrank[b])
        np.minimum.at(primary, b, hubrank[a])
        tail = perm[H:]
        perm = np.concatenate([perm[:H], tail[np.argsort(primary[tail], kind="stable")]])
    inv = np.empty(V, np.int64)
    inv[perm] = np.arange(V)
    rows = np.concatenate([inv[a], inv[b]])
    cols = np.concatenate([inv[b], inv[a]])
    eids = np.concatenate([e, e])
    ws = np.concatenate([w, w])
    o = np.lexsort((eids, cols, rows))
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=V))])
    g = sp.csr_matrix((w, (a, b)), shape=(V, V))
    d0 = dijkstra(g, directed=False, indices=[int(perm[0])])[0]
    pot = d0[perm]
    return dict(perm=perm, rowptr=rowptr, rows=rows[o], col=cols[o], w=ws[o], pot=pot, V=V)


@pytest.mark.parametrize("n_routers,n_poi,n_edges", [(3000, 150, 30000), (40000, 400, 250000)])
def test_gpu_prep_matches_restatement(n_routers, n_poi, n_edges):
    top = sa.Topology.synthetic(seed=41, n_routers=n_routers, n_poi=n_poi, n_edges=n_edges)
    assert top is not None and not top.is_complete
    got = top.export_csr()
    ref = restate(top)
    V = ref["V"]
    assert np.array_equal(got["perm"], ref["perm"])
    assert np.array_equal(got["rowptr"].astype(np.int64), ref["rowptr"])
    assert np.array_equal(got["col"].astype(np.int64), ref["col"])
    # pi: bit-identical to scipy's distances (unique monotone-rounding fixpoint)
    assert np.array_equal(got["pot"].view(np.uint64), ref["pot"].view(np.uint64))
    # h0 tree: argmin (d(u), u) over the tight edges (u, v) with d(u) < d(v)
    pot, rows, col, w = ref["pot"], ref["rows"], ref["col"], ref["w"]
    tight = (pot[col] < pot[rows]) & (pot[col] + w == pot[rows])
    r, u = rows[tight], col[tight]
    o = np.lexsort((u, pot[u], r))
    r, u = r[o], u[o]
    first = np.ones(len(r), bool)
    first[1:] = r[1:] != r[:-1]
    want = np.full(V, 0xFFFFFFFF, np.uint64)
    want[r[first]] = u[first]
    assert np.array_equal(got["tree_parent"].astype(np.uint64), want)
    assert want[0] == 0xFFFFFFFF and np.count_nonzero(want == 0xFFFFFFFF) == 1
    st = top.stats()
    assert st["csr_h0_rounds"] > 0


def test_attach_time_preparation_matches_build_time():
    """Option prepare_on_attach (default on): device init + graph preparation start in a
    background thread at the first attach and the first build waits for it under the build lock.
    The table must be bit-identical to a build that prepares everything itself, and only the
    former reports a background preparation."""
    tables = []
    for on in (1, 0):
        top = sa.Topology.synthetic(seed=43, n_routers=40000, n_poi=400, n_edges=250000)
        top.set_option("prepare_on_attach", on)
        top.synth_packets(5, 2000, 10, 10**9, 10**7)
        time.sleep(3.0)  # let the background preparation win the build lock (it takes ~0.2 s)
        A, lat, rel, hops = top.table()
        st = top.stats()
        if on:
            assert st["attach_prep_ms"] > 0.0 and st["csr_ms"] == 0.0
        else:
            assert st["attach_prep_ms"] == 0.0 and st["csr_ms"] > 0.0
        tables.append((np.asarray(A), lat.view(np.uint64), rel.view(np.uint64), hops))
    for x, y in zip(*tables):
        assert np.array_equal(x, y)
