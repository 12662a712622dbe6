"""CPU tests: pin the oracle (the checker) before trusting it.

Anchors available for this path: glibc's own rand_r (the reference's RNG
dependency), the reference's tcp test topologies (1 vertex, loss 0 / 0.25), the survey's
independently computed seed chain for config 1, and scipy's Dijkstra for distances.  igraph's
parent choice on ties is "parity unpinned" (igraph is absent).
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, bundled_topology

LIBC = ctypes.CDLL("libc.so.6")


def test_rand_r_matches_glibc():
    for seed in (0, 1, 12345, 0xFFFFFFFF, 20261015, 476707713):
        s = ctypes.c_uint(seed)
        st = seed
        for _ in range(2000):
            want = LIBC.rand_r(ctypes.byref(s))
            got, st = oracle.rand_r(st)
            assert got == want and st == s.value


def test_seed_chain_config1_matches_survey():
    """slave seed 476707713, node seeds 679019682 / 59974537, first draws
    0.27939451731713233 / 0.92984414563041373 -> poi-1 / poi-2."""
    d = json.load(open(os.path.join(GOLDEN, "c1_simple.json")))
    assert d["slave_seed"] == 476707713
    assert [h["node_seed"] for h in d["hosts"]] == [679019682, 59974537]
    assert d["hosts"][0]["first_draw"] == 0.27939451731713233
    assert d["hosts"][1]["first_draw"] == 0.92984414563041373
    assert [h["vertex_id"] for h in d["hosts"]] == ["poi-1", "poi-2"]
    assert d["lat"] == [[20.0, 50.0], [50.0, 20.0]] and d["global_min"] == 20.0
    # recompute from scratch
    g = oracle.OGraph.from_graphml(bundled_topology("topology.simple"))
    a, lat, rel, hops = g.table([0, 1])
    assert lat.tolist() == d["lat"] and rel.tolist() == d["rel"]


@pytest.mark.parametrize("name", ["lossless", "lossy"])
def test_tcp_test_topologies(name):
    """The reference's only topology fixtures (src/test/tcp/*.test.shadow.config.xml:14-26)."""
    d = json.load(open(os.path.join(GOLDEN, "tcp_1vertex.json")))[name]
    g = oracle.OGraph.from_graphml(d["graphml"].encode())
    assert g.is_complete() and g.V == 1
    lat, rel = g.complete_pairs([0], [0])
    assert lat[0] == 50.0 == d["latency"]
    assert rel[0] == (0.75 if name == "lossy" else 1.0) == d["reliability"]


def test_bundled_graph_facts():
    """Appendix B: V, E, self loops, completeness of the three bundled topologies."""
    facts = {"topology.simple": (2, 3), "topology": (183, 16836), "topology.plab": (303, 46056)}
    for name, (V, E) in facts.items():
        g = oracle.OGraph.from_graphml(bundled_topology(name))
        assert (g.V, g.E) == (V, E)
        assert g.is_complete() and g.is_strongly_connected()
        assert int((g.eu == g.ev).sum()) == V


@pytest.mark.parametrize("name", ["topology", "topology.plab"])
def test_bundled_tables_golden(name):
    import hashlib
    d = json.load(open(os.path.join(GOLDEN, "bundled_tables.json")))[name]
    g = oracle.OGraph.from_graphml(bundled_topology(name))
    st = 1
    verts = []
    for v in range(g.V):
        st = (st * 1103515245 + 12345) & 0xFFFFFFFF
        vv, _, _ = oracle.attach_vertex(g.vattrs, st, geocode_hint=g.vattrs["geocode"][v])
        verts.append(vv)
    a, lat, rel, hops = g.table(verts)
    assert len(a) == d["A"]
    assert hashlib.sha256(lat.tobytes()).hexdigest() == d["sha256_lat"]
    assert hashlib.sha256(rel.tobytes()).hexdigest() == d["sha256_rel"]
    for i, j, l, r in d["samples"]:
        assert lat[i, j] == l and rel[i, j] == r


@pytest.mark.parametrize("tag", ["real", "int"])
def test_synthetic_rows_golden_and_scipy(tag):
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    z = np.load(os.path.join(GOLDEN, "synth_%s.npz" % tag))
    g = oracle.OGraph(int(z["V"]), z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    lat, rel, hops = g.source_rows(z["sources"], z["targets"])
    assert np.array_equal(lat, z["lat"]) and np.array_equal(rel, z["rel"])
    assert np.array_equal(hops, z["hops"])
    m = z["eu"] != z["ev"]
    A = sp.coo_matrix((z["elat"][m], (z["eu"][m], z["ev"][m])), shape=(g.V, g.V)).tocsr()
    for i, s in enumerate(z["sources"]):
        d, pv, pe, rank = g.dijkstra(int(s))
        assert np.array_equal(d, z["dist"][i]) and np.array_equal(pv, z["parent"][i])
        ds = dijkstra(A, directed=False, indices=int(s))
        assert np.array_equal(d, ds)                     # distances: unique fixpoint
        other = z["targets"] != s                        # self pair = the self loop (A.4)
        assert np.array_equal(lat[i][other], d[z["targets"][other]])  # latency == dist (A.3)
    if tag == "real":
        assert z["tied_vertices"].sum() == 0
    else:
        assert z["tied_vertices"].sum() > 0


def test_parent_rule_reproduces_heap_parents():
    """A.3: parent(v) = argmin (d[u], popRank(u)) over candidates fl(d[u]+w) == d[v]."""
    z = np.load(os.path.join(GOLDEN, "synth_int.npz"))
    g = oracle.OGraph(int(z["V"]), z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    for s in z["sources"][:6]:
        d, pv, pe, rank = g.dijkstra(int(s))
        for x in range(g.V):
            if x == s or d[x] < 0:
                continue
            cands = []
            for i in range(g.inc_ptr[x], g.inc_ptr[x + 1]):
                e = g.inc_eid[i]
                y = g.efrom[e] if g.efrom[e] != x else g.eto[e]
                if y != x and d[y] >= 0 and d[y] + g.elat[e] == d[x]:
                    cands.append((d[y], rank[y], y))
            assert min(cands)[2] == pv[x]


def test_packets_golden():
    z = np.load(os.path.join(GOLDEN, "packets.npz"))
    t, dl, st = oracle.route_packets(z["lat"], z["rel"], z["payload"], z["state"], z["now"],
                                     int(z["jump"]), 1)
    assert np.array_equal(t, z["time_clamp"]) and np.array_equal(dl, z["delivered"])
    assert np.array_equal(st, z["state_out"])
    t2, _, _ = oracle.route_packets(z["lat"], z["rel"], z["payload"], z["state"], z["now"],
                                    int(z["jump"]), 0)
    assert np.array_equal(t2, z["time_noclamp"])
    # control packets are never dropped; drops only where chance > rel
    assert np.all(dl[z["payload"] == 0] == 1)
    assert np.all(dl[z["rel"] == 1.0] == 1)


def test_lazy_cache_first_rooted_wins():
    """K3: (a,b) after rooting b returns row b's entry; min trajectory follows stored pairs."""
    z = np.load(os.path.join(GOLDEN, "synth_real.npz"))
    g = oracle.OGraph(int(z["V"]), z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    t = oracle.OracleTopology(g)
    ips = []
    for k, v in enumerate((1400, 1401, 1402)):
        t.virtual_ip[100 + k] = v
        ips.append(100 + k)
    l_ba = t.get_latency(ips[1], ips[0])          # roots vertex 1401
    assert 1401 in t.cache and 1400 not in t.cache
    l_ab = t.get_latency(ips[0], ips[1])          # served from row 1401 (reverse entry)
    assert l_ab == l_ba and 1400 not in t.cache
    assert t.minimum_path_latency == min(v[0] for v in t.cache[1401].values())


def test_master_min_jump():
    assert oracle.master_min_jump(0) == 10_000_000
    assert oracle.master_min_jump(7.9) == 7_000_000
    assert oracle.master_min_jump(7.9, runahead_ms=9) == 9_000_000


def _scipy_rows(V, eu, ev, elat, eloss, vloss, sources, targets):
    """Latency / reliability / hops of every (source, target) pair from scipy's shortest-path
    TREE (dijkstra with return_predecessors) -- an implementation independent of the oracle's
    igraph restatement.  On a tie-free graph the shortest paths are unique, so any correct
    Dijkstra returns igraph's parents; reliability then follows shd-topology.c:561-671 (A.4)."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    m = eu != ev
    A = sp.coo_matrix((elat[m], (eu[m], ev[m])), shape=(V, V)).tocsr()
    eidx = {}
    for e in np.nonzero(m)[0]:
        eidx.setdefault((min(eu[e], ev[e]), max(eu[e], ev[e])), e)
    dist, pred = dijkstra(A, directed=False, indices=np.asarray(sources), return_predecessors=True)
    out_lat = np.zeros((len(sources), len(targets)))
    out_rel = np.zeros_like(out_lat)
    out_hops = np.zeros((len(sources), len(targets)), np.int64)
    for i, s in enumerate(sources):
        for j, t in enumerate(targets):
            if t == s:
                continue
            path = [int(t)]
            while path[-1] != s:
                path.append(int(pred[i, path[-1]]))
            path.reverse()
            rel = 1.0
            rel *= (1.0 - vloss[s])
            rel *= (1.0 - vloss[t])
            for a, b in zip(path[:-1], path[1:]):
                rel *= (1.0 - eloss[eidx[(min(a, b), max(a, b))]])
            out_lat[i, j] = dist[i, t]
            out_rel[i, j] = rel
            out_hops[i, j] = len(path) - 1
    return out_lat, out_rel, out_hops


def test_oracle_paths_pinned_by_scipy_on_tie_free_graph():
    """with continuous latencies shortest paths are unique, so scipy's
    predecessor tree must equal the oracle's igraph parents -- and the oracle's hops and
    reliability (the golden rows) must equal the ones rebuilt from scipy's tree.  This pins the
    SSSP branch independently of the oracle's own restatement where no ties exist; tie handling
    (integer latencies) stays parity-unpinned."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    z = np.load(os.path.join(GOLDEN, "synth_real.npz"))
    V = int(z["V"])
    g = oracle.OGraph(V, z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    m = z["eu"] != z["ev"]
    A = sp.coo_matrix((z["elat"][m], (z["eu"][m], z["ev"][m])), shape=(V, V)).tocsr()
    for s in z["sources"]:
        d, pv, pe, rank = g.dijkstra(int(s))
        ds, pred = dijkstra(A, directed=False, indices=int(s), return_predecessors=True)
        reached = (d >= 0) & (np.arange(V) != s)
        assert np.array_equal(pv[reached], pred[reached])
    lat, rel, hops = _scipy_rows(V, z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"],
                                 z["sources"], z["targets"])
    other = z["targets"][None, :] != z["sources"][:, None]
    assert np.array_equal(lat[other], z["lat"][other])
    assert np.array_equal(rel[other].view(np.uint64), z["rel"][other].view(np.uint64))
    assert np.array_equal(hops[other], z["hops"][other])


def test_vectorised_scipy_helper_matches_golden_rows():
    """tests/helpers.scipy_rows (the full-size C4 GPU test's independent pin: scipy predecessor
    trees + the reference helper, vectorised over targets) reproduces the oracle's golden rows of
    the tie-free graph bit for bit, self pairs included."""
    from helpers import scipy_rows
    z = np.load(os.path.join(GOLDEN, "synth_real.npz"))
    graph = (int(z["V"]), z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    lat, rel, hops = scipy_rows(graph, z["sources"], z["targets"])
    assert np.array_equal(lat.view(np.uint64), z["lat"].view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), z["rel"].view(np.uint64))
    assert np.array_equal(hops, z["hops"])
