"""Shared test helpers: build the same topology for the product (HIP) and the oracle (CPU)."""
import os
import tempfile

import numpy as np

import oracle
import shadow_amd as sa
from conftest import bundled_topology


def bundled_pair(name):
    data = bundled_topology(name)
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    return top, g


def synthetic_pair(seed=7, n_routers=2000, n_poi=100, n_edges=20000, integer=False):
    top = sa.Topology.synthetic(seed=seed, n_routers=n_routers, n_poi=n_poi, n_edges=n_edges,
                                integer_latency=integer)
    assert top is not None
    fd, path = tempfile.mkstemp(suffix=".graphml.xml")
    os.close(fd)
    try:
        top.write_graphml(path)
        g = oracle.OGraph.from_graphml(path)
    finally:
        os.unlink(path)
    return top, g


def host_ip(k):
    return sa.ip_to_network("11.%d.%d.%d" % ((k >> 16) & 255, (k >> 8) & 255, k & 255))


def attach_hosts(top, g, n_hosts, seed=1, type_hints=None, geo_hints=None):
    """Attach n hosts to both the product and the oracle topology with identical RNG streams.
    Returns (ips, vertices)."""
    otop = oracle.OracleTopology(g)
    ips, verts = [], []
    st = seed
    for k in range(n_hosts):
        st = (st * 1103515245 + 12345) & 0xFFFFFFFF  # distinct per-host seeds
        th = type_hints[k % len(type_hints)] if type_hints else None
        gh = geo_hints[k] if geo_hints else None
        ip = host_ip(k + 1)
        v1, s1 = top.attach_ip(ip, st, typeHint=th, geocodeHint=gh)
        v2, s2 = otop.attach(ip, st, type_hint=th, geocode_hint=gh)
        assert v1 == v2 and s1 == s2, (k, v1, v2, s1, s2)
        ips.append(ip)
        verts.append(v1)
    return otop, ips, verts


def oracle_table(g, verts):
    return g.table(verts)


def rel_close(a, b, tol=1e-12):
    a = np.asarray(a)
    b = np.asarray(b)
    return np.all(np.abs(a - b) <= tol * np.maximum(np.abs(b), 1e-300))


_KEYS = ('<key attr.name="packetloss" attr.type="double" for="edge" id="d9" />'
         '<key attr.name="jitter" attr.type="double" for="edge" id="d8" />'
         '<key attr.name="latency" attr.type="double" for="edge" id="d7" />'
         '<key attr.name="type" attr.type="string" for="node" id="d5" />'
         '<key attr.name="bandwidthup" attr.type="int" for="node" id="d4" />'
         '<key attr.name="bandwidthdown" attr.type="int" for="node" id="d3" />'
         '<key attr.name="geocode" attr.type="string" for="node" id="d2" />'
         '<key attr.name="ip" attr.type="string" for="node" id="d1" />'
         '<key attr.name="packetloss" attr.type="double" for="node" id="d0" />')


def graphml_doc(nodes, edges, directed=False):
    """GraphML text in the bundled files' key schema.  nodes: (id, type, loss);
    edges: (src, dst, latency, loss)."""
    out = ['<?xml version="1.0" encoding="utf-8"?><graphml '
           'xmlns="http://graphml.graphdrawing.org/xmlns">', _KEYS,
           '<graph edgedefault="%s">' % ("directed" if directed else "undirected")]
    for nid, typ, loss in nodes:
        out.append('<node id="%s"><data key="d0">%r</data><data key="d1">0.0.0.0</data>'
                   '<data key="d2">US</data><data key="d3">10240</data>'
                   '<data key="d4">10240</data><data key="d5">%s</data></node>'
                   % (nid, float(loss), typ))
    for a, b, lat, loss in edges:
        out.append('<edge source="%s" target="%s"><data key="d7">%r</data>'
                   '<data key="d8">0</data><data key="d9">%r</data></edge>'
                   % (a, b, float(lat), float(loss)))
    out.append("</graph></graphml>")
    return "".join(out).encode()


def random_topology_graphml(n_routers=600, n_poi=60, extra=2400, seed=3, integer=False,
                            directed=False, parallel=0, lat_scale=1):
    """A connected router graph (a cycle, both directions when directed, plus `extra` random
    edges), poi vertices with an uplink (a pair of opposite edges when directed) and a self loop.
    `parallel` extra edges duplicate existing router edges with other latencies (multigraph).
    Router latencies are U{1..100} x lat_scale (integer) or U[1, 100)."""
    rng = np.random.default_rng(seed)
    lat = ((lambda: int(rng.integers(1, 101)) * lat_scale) if integer
           else (lambda: rng.uniform(1, 100)))
    nodes = [("pop-%d" % i, "pop", 0.0) for i in range(n_routers)]
    nodes += [("poi-%d" % k, ("client", "relay", "server")[k % 3], rng.uniform(0, 0.05))
              for k in range(n_poi)]
    edges = []
    for i in range(n_routers):
        j = (i + 1) % n_routers
        edges.append(("pop-%d" % i, "pop-%d" % j, lat(), rng.uniform(0, 0.01)))
        if directed:
            edges.append(("pop-%d" % j, "pop-%d" % i, lat(), rng.uniform(0, 0.01)))
    seen = set()
    while len(seen) < extra:
        a, b = (int(x) for x in rng.integers(0, n_routers, 2))
        key = (a, b) if directed else (min(a, b), max(a, b))
        if a == b or abs(a - b) in (1, n_routers - 1) or key in seen:
            continue
        seen.add(key)
        edges.append(("pop-%d" % a, "pop-%d" % b, lat(), rng.uniform(0, 0.01)))
    for _ in range(parallel):
        a, b, _, _ = edges[int(rng.integers(0, len(edges)))]
        edges.append((a, b, lat(), rng.uniform(0, 0.01)))
    for k in range(n_poi):
        r = "pop-%d" % int(rng.integers(0, n_routers))
        edges.append(("poi-%d" % k, r, 5.0, 0.0))
        if directed:
            edges.append((r, "poi-%d" % k, float(lat()), 0.0))
        edges.append(("poi-%d" % k, "poi-%d" % k, 1.0, 0.0))
    order = rng.permutation(len(edges))  # edge ids not grouped by vertex
    return graphml_doc(nodes, [edges[i] for i in order], directed)


def scipy_rows(graph, srcs, targets, directed=False):
    """The per-target helper (shd-topology.c:561-671) over scipy's shortest-path trees, an
    implementation independent of the oracle: scipy.sparse.csgraph.dijkstra with predecessors on
    the undirected non-loop graph.  latency = scipy's distance (the same left-to-right f64 sums
    from the source), hops = the predecessor chain's length, reliability = ((1 * (1 - vloss[s]))
    * (1 - vloss[t])) * prod(1 - loss(e)) in path order from the source; the self pair is the
    self loop (latency 0 + its latency, reliability (1 - vloss) * (1 - loss), 1 hop).  directed:
    the arcs as given (igraph mode OUT)."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import dijkstra
    V, eu, ev, elat, eloss, vloss = graph
    eu, ev = np.asarray(eu, np.int64), np.asarray(ev, np.int64)
    elat, eloss = np.asarray(elat, np.float64), np.asarray(eloss, np.float64)
    vloss = np.asarray(vloss, np.float64)
    nl = eu != ev
    if directed:
        r, c, wl, wo = eu[nl], ev[nl], elat[nl], eloss[nl]
    else:
        r = np.concatenate([eu[nl], ev[nl]])
        c = np.concatenate([ev[nl], eu[nl]])
        wl = np.concatenate([elat[nl], elat[nl]])
        wo = np.concatenate([eloss[nl], eloss[nl]])
    W = sp.csr_matrix((wl, (r, c)), shape=(V, V))
    Lm = sp.csr_matrix((wo, (r, c)), shape=(V, V))
    # no parallel edges (the csr would sum them) and no zero latency (scipy drops zeros)
    assert W.nnz == len(r) and bool((W.data > 0).all())
    # self loops: the first (lowest edge id) per vertex, as igraph_get_eid
    selfLat = np.full(V, np.nan)
    selfLoss = np.zeros(V)
    li = np.nonzero(~nl)[0][::-1]  # assigned last-to-first: the lowest edge id wins
    selfLat[eu[li]] = elat[li]
    selfLoss[eu[li]] = eloss[li]
    dist, pred = dijkstra(W, directed=directed, indices=np.asarray(srcs), return_predecessors=True)
    targets = np.asarray(targets, np.int64)
    A = len(targets)
    lat = np.empty((len(srcs), A))
    rel = np.empty((len(srcs), A))
    hops = np.zeros((len(srcs), A), np.int64)
    for i, s in enumerate(srcs):
        lat[i] = dist[i, targets]
        cur = targets.copy()
        losses = []
        act = cur != s
        while act.any():
            p = pred[i, cur]
            p = np.where(act, p, cur)
            assert bool((p[act] >= 0).all())
            lo = np.zeros(A)
            lo[act] = np.asarray(Lm[p[act], cur[act]]).ravel()
            losses.append(lo)
            hops[i] += act
            cur = np.where(act, p, cur)
            act = cur != s
        rr = (1.0 * (1.0 - vloss[s])) * (1.0 - vloss[targets])
        for k in range(len(losses) - 1, -1, -1):  # the edge at depth k from the target
            rr = np.where(k < hops[i], rr * (1.0 - losses[k]), rr)
        rel[i] = rr
        lat[i] = np.where(lat[i] == 0.0, 1.0, lat[i])  # the helper's zero-latency rule
        selfc = targets == s
        lat[i, selfc] = 0.0 + selfLat[s]
        rel[i, selfc] = (1.0 * (1.0 - vloss[s])) * (1.0 - selfLoss[s])
        hops[i, selfc] = 1
    return lat, rel, hops
