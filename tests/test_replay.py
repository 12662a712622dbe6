"""GPU parity of the exact heap replay (topo_replay.hip) against the igraph-0.7 restatement.

The replay runs igraph_get_shortest_paths_dijkstra with its two-way heap operation for operation
(oracle/oracle.c:146-305 is the restated spec), so on integer latencies -- where many vertices
have several candidate parents at the same d[u] and igraph's pop order decides -- every
distance AND every parent must equal the oracle's.  Through the table path this resolves the rows
the batch kernel flags (ambiguous_pairs), directed topologies and multigraphs.
"""
import numpy as np
import pytest

import oracle
import shadow_amd as sa
from helpers import attach_hosts, graphml_doc, random_topology_graphml, synthetic_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("integer,int_keys", [(True, 1), (True, 0), (False, 1)])
def test_replay_full_dijkstra_parents_match_oracle(integer, int_keys):
    """Full Dijkstra (no early exit): dist bit-exact and the parent of EVERY vertex equal to the
    oracle heap's, ties included -- on the u32-key heap (integer latencies) and the f64 one."""
    top, g = synthetic_pair(seed=11, n_routers=3000, n_poi=150, n_edges=30000, integer=integer)
    top.set_option("replay_int_keys", int_keys)
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    srcs = sorted(set(verts))[:4] + [0, g.V // 2]
    nties = 0
    for s in srcs:
        d, p = top.replay_source(s, full=True)
        od, opv, _, _ = g.dijkstra(s)
        assert np.array_equal(d.view(np.uint64), od.view(np.uint64)), s
        assert np.array_equal(p, opv), (s, int(np.sum(p != opv)))
        nties += int(np.sum(g.parent_ties(od, s) >= 2))
    if integer:
        assert nties > 50  # the case the replay exists for


@pytest.mark.parametrize("int_keys", [1, 0])
def test_replay_deep_heap_matches_oracle(int_keys):
    """A graph large enough (V > 2^15) that the heap grows well past its 9 LDS levels into the HBM
    levels -- in a SHD_RP_BLOCKED build the blocked sink-round layout of levels 9-13
    (topo_replay.hip RpHeap::phys) and position-major levels below: full Dijkstra from three
    sources, distances and every parent equal to the oracle's."""
    top, g = synthetic_pair(seed=21, n_routers=40000, n_poi=200, n_edges=300000, integer=True)
    top.set_option("replay_int_keys", int_keys)
    attach_hosts(top, g, 200, type_hints=["client", "relay"])
    for s in [0, g.V // 3, g.V - 1]:
        d, p = top.replay_source(s, full=True)
        od, opv, _, _ = g.dijkstra(s)
        assert np.array_equal(d.view(np.uint64), od.view(np.uint64)), s
        assert np.array_equal(p, opv), (s, int(np.sum(p != opv)))


def test_replay_early_exit_matches_oracle():
    """The reference's early exit (all attached targets popped): every vertex popped before it
    has the oracle's parent."""
    top, g = synthetic_pair(seed=12, n_routers=2500, n_poi=120, n_edges=25000, integer=True)
    otop, ips, verts = attach_hosts(top, g, 200, type_hints=["client", "relay"])
    targets = np.asarray(sorted(set(verts)), np.int32)
    for s in targets[:5]:
        d, p = top.replay_source(int(s), full=False)
        od, opv, _, rank = g.dijkstra(int(s), targets)
        popped = rank >= 0
        assert popped[targets].all()
        assert np.array_equal(d[popped].view(np.uint64), od[popped].view(np.uint64))
        assert np.array_equal(p[popped], opv[popped])


@pytest.mark.parametrize("fill", [8, 1])
def test_integer_ties_table_bit_exact(fill):
    """Integer latencies U{1..100}: every pair of the table -- hops and reliability included --
    bit-exact against the oracle; the tie rows went through the replay."""
    top, g = synthetic_pair(seed=11, n_routers=3000, n_poi=150, n_edges=30000, integer=True)
    top.set_option("batch_fill", fill)
    top.set_option("tie_dense", 0)  # the batch kernel + flagged-row replay path (no tie probe)
    otop, ips, verts = attach_hosts(top, g, 400, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert st["errors"] == 0
    assert st["ambiguous_pairs"] > 0 and st["replay_rows"] > 0
    assert st["replay_pops"] > 0 and st["replay_ms"] > 0
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert top.getMinimumLatency() == olat.min()


def test_tie_replay_off_reports_only():
    """tie_replay = 0: the batch kernel's table stands (latencies exact), nothing replayed."""
    top, g = synthetic_pair(seed=11, n_routers=3000, n_poi=150, n_edges=30000, integer=True)
    top.set_option("tie_replay", 0)
    otop, ips, verts = attach_hosts(top, g, 400, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert st["ambiguous_pairs"] > 0 and st["replay_rows"] == 0
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))


def test_replay_all_equals_oracle_continuous():
    """replay_all: the replay alone builds the whole table (continuous latencies)."""
    top, g = synthetic_pair(seed=5, n_routers=1500, n_poi=80, n_edges=15000)
    top.set_option("replay_all", 1)
    otop, ips, verts = attach_hosts(top, g, 200, type_hints=["client", "relay"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert st["replay_rows"] == len(a) and st["errors"] == 0
    assert st["replay_int_keys"] == 0  # continuous latencies: f64 keys
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))


@pytest.mark.parametrize("scale,int_keys", [(60000, 1), (1 << 23, 0)])
def test_replay_int_key_bound(scale, int_keys):
    """u32 heap keys only while V x max latency < 2^32 - 1 (660 x 100 x 60000 = 3.96e9 fits;
    x 2^23 does not and falls back to f64 keys); every pair bit-exact either way."""
    data = random_topology_graphml(n_routers=600, n_poi=60, extra=2400, seed=4, integer=True,
                                   lat_scale=scale)
    top = sa.Topology.from_buffer(data)
    top.set_option("replay_all", 1)
    g = oracle.OGraph.from_graphml(data)
    otop, ips, verts = attach_hosts(top, g, 100, type_hints=["client", "relay"])
    st = _table_bit_exact(top, g, verts)
    assert st["errors"] == 0 and st["replay_rows"] == len(top.attached_vertices())
    assert st["replay_int_keys"] == int_keys


@pytest.mark.parametrize("integer,n_routers,extra,mode", [
    (False, 500, 2500, "batch"), (True, 500, 2500, "batch"),
    (False, 6000, 30000, "batch"), (True, 6000, 30000, "batch"),
    (False, 500, 2500, "replay_all"), (True, 500, 2500, "replay_all")])
def test_directed_topology_table(integer, n_routers, extra, mode):
    """Directed non-complete topology (igraph mode OUT, shd-topology.c:153,762-763): the batch
    kernel relaxes the out-rows and finds each vertex's parent among its in-rows (DevCSR
    rowptr_in), rows crossing a tie go through the replay (mode "batch"); or the replay alone
    builds every row ("replay_all").  Bit-exact against the oracle either way.  6,000 routers put
    most vertices past the LDS hubs, so the tail paths (in-row scans, improver hints, tree walks)
    run too.  Getters answer forward rows only (no reverse lookup for directed graphs,
    shd-topology.c:896-898)."""
    data = random_topology_graphml(n_routers=n_routers, n_poi=50, extra=extra, seed=7,
                                   integer=integer, directed=True)
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    assert top.is_directed and g.directed and not top.is_complete
    if mode == "replay_all":
        top.set_option("replay_all", 1)
    else:
        top.set_option("tie_dense", 0)  # the batch kernel + flagged-row replay (no tie probe)
    otop, ips, verts = attach_hosts(top, g, 120, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert st["errors"] == 0
    if mode == "replay_all":
        assert st["replay_rows"] == len(a)
    else:
        assert st["sssp_kernel_ms"] > 0  # the batch kernel ran
        if not integer:
            assert st["replay_rows"] == 0  # no ties: every row is the batch kernel's
    assert not np.array_equal(lat, lat.T)  # really directed
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    # lazy getters against the reference cache (forward rows only)
    rng = np.random.default_rng(2)
    for _ in range(200):
        x, y = (int(v) for v in rng.choice(ips, 2))
        assert top.latency_ip(x, y) == otop.get_latency(x, y)
        assert top.reliability_ip(x, y) == otop.get_reliability(x, y)
    assert top.lazyMinimumLatency() == otop.minimum_path_latency


@pytest.mark.parametrize("directed", [False, True])
def test_multigraph_table(directed):
    """Parallel edges with different latencies: the reference sums the igraph_get_eid edge of
    each hop (lowest edge id, as the oracle); every row goes through the replay."""
    data = random_topology_graphml(n_routers=400, n_poi=40, extra=1600, seed=9, integer=True,
                                   directed=directed, parallel=300)
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    otop, ips, verts = attach_hosts(top, g, 80, type_hints=["client", "relay"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert st["errors"] == 0 and st["replay_rows"] == len(a)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))


def _table_bit_exact(top, g, verts):
    a, lat, rel, hops = top.table()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    return top.stats()


@pytest.mark.parametrize("landmark,int_keys", [(1, 1), (0, 1), (1, 0)])
def test_tie_dense_replay_landmark_skip(landmark, int_keys):
    """tie_dense = 1: no batch kernel, every row through the replay; the replay's landmark skip
    (relaxations into vertices d(h0) + pi(t) < du proves popped: their record is not read) on or
    off, u32 or f64 heap keys -- every pair bit-exact against the oracle either way."""
    top, g = synthetic_pair(seed=11, n_routers=3000, n_poi=150, n_edges=30000, integer=True)
    top.set_option("tie_dense", 1)
    top.set_option("replay_landmark", landmark)
    top.set_option("replay_int_keys", int_keys)
    otop, ips, verts = attach_hosts(top, g, 400, type_hints=["client", "relay", "server"])
    st = _table_bit_exact(top, g, verts)
    assert st["tie_dense"] == 1 and st["errors"] == 0
    assert st["replay_int_keys"] == int_keys
    assert st["replay_rows"] == len(top.attached_vertices())
    assert st["ambiguous_pairs"] == 0  # the batch kernel did not run
    if landmark:
        assert st["replay_skips"] > st["replay_pops"]  # several per pop on this graph
    else:
        assert st["replay_skips"] == 0


def test_tie_dense_auto_switch():
    """tie_dense auto (-1).  The first batched build of an integer-latency topology probes 64
    sample rows with the batch kernel: if >= 90 % of them cross a d-tied parent the topology is
    tie-dense before the full launch and every row goes straight to the heap replay (no batch
    kernel over the table); otherwise a build that replays >= 90 % of >= 64 rows switches the
    later builds.  Every build's rows are bit-identical (and equal the oracle's)."""
    import torch
    top, g = synthetic_pair(seed=11, n_routers=3000, n_poi=300, n_edges=30000, integer=True)
    otop, ips, verts = attach_hosts(top, g, 800, type_hints=["client", "relay", "server"])
    A = len(top.attached_vertices())
    assert A >= 128  # the probe needs twice its sample (A = 191 here)
    outs, sts = [], []
    for _ in range(2):
        lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
        hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
        top.build_rows_into(0, A, lr, hp)
        torch.cuda.synchronize()
        outs.append((lr.cpu().numpy(), hp.cpu().numpy()))
        sts.append(top.stats())
    st0, st1 = sts
    assert st0["tie_probe_rows"] == 64 and st1["tie_probe_rows"] == 0  # once per topology
    probe_dense = st0["tie_probe_flagged"] * 10 >= 64 * 9
    assert st0["tie_dense"] == (1 if probe_dense else 0)
    if probe_dense:
        # decided before the full launch: every row replayed, none flagged by a batch launch
        assert st0["replay_rows"] == A and st0["ambiguous_pairs"] == 0
    dense = probe_dense or st0["replay_rows"] * 10 >= A * 9
    assert st1["tie_dense"] == (1 if dense else 0)
    if dense:
        assert st1["replay_rows"] == A and st1["ambiguous_pairs"] == 0
    assert np.array_equal(outs[0][0].view(np.uint64), outs[1][0].view(np.uint64))
    assert np.array_equal(outs[0][1], outs[1][1])
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(outs[1][0][..., 0].view(np.uint64), olat.view(np.uint64))


def _one_way_regions_graphml(back_lat=5000.0, seed=11, with_back=True):
    """A directed topology whose two side regions hang off a strongly connected core almost one
    way: the sink region is entered by many cheap arcs and left by ONE arc of latency `back_lat`,
    the source region left by many cheap arcs and entered by ONE such arc.  With the two arcs the
    graph is strongly connected (the reference's requirement, shd-topology.c:134-151); without
    them it is not.  Poi sit in the core and in both regions."""
    rng = np.random.default_rng(seed)
    core, side = 300, 120
    nodes = [("pop-%d" % i, "pop", 0.0) for i in range(core + 2 * side)]
    edges, seen = [], set()

    class _Arcs(list):  # no parallel arcs (a multigraph would send every row to the replay)
        def append(self, e):
            if (e[0], e[1]) not in seen:
                seen.add((e[0], e[1]))
                list.append(self, e)
    edges = _Arcs()
    for i in range(core):  # core: bidirectional cycle + random arcs
        j = (i + 1) % core
        edges.append(("pop-%d" % i, "pop-%d" % j, rng.uniform(1, 100), rng.uniform(0, 0.01)))
        edges.append(("pop-%d" % j, "pop-%d" % i, rng.uniform(1, 100), rng.uniform(0, 0.01)))
    for _ in range(900):
        a, b = (int(x) for x in rng.integers(0, core, 2))
        if a != b:
            edges.append(("pop-%d" % a, "pop-%d" % b, rng.uniform(1, 100), rng.uniform(0, 0.01)))
    sink = list(range(core, core + side))
    src = list(range(core + side, core + 2 * side))
    for reg in (sink, src):  # each region: a bidirectional chain + random internal arcs
        for a, b in zip(reg[:-1], reg[1:]):
            edges.append(("pop-%d" % a, "pop-%d" % b, rng.uniform(1, 100), rng.uniform(0, 0.01)))
            edges.append(("pop-%d" % b, "pop-%d" % a, rng.uniform(1, 100), rng.uniform(0, 0.01)))
        for _ in range(200):
            a, b = (int(x) for x in rng.choice(reg, 2))
            if a != b:
                edges.append(("pop-%d" % a, "pop-%d" % b, rng.uniform(1, 100), rng.uniform(0, 0.01)))
    for _ in range(60):  # cheap one-way arcs: core -> sink region, source region -> core
        c = int(rng.integers(0, core))
        edges.append(("pop-%d" % c, "pop-%d" % int(rng.choice(sink)), rng.uniform(1, 100), 0.0))
        edges.append(("pop-%d" % int(rng.choice(src)), "pop-%d" % c, rng.uniform(1, 100), 0.0))
    if with_back:  # the only ways back
        edges.append(("pop-%d" % sink[-1], "pop-0", back_lat, 0.0))
        edges.append(("pop-0", "pop-%d" % src[0], back_lat, 0.0))
    n_poi = 45
    for k in range(n_poi):
        pool = (range(core), sink, src)[k % 3]
        r = "pop-%d" % int(rng.choice(list(pool)))
        nodes.append(("poi-%d" % k, ("client", "relay", "server")[k % 3], rng.uniform(0, 0.05)))
        edges.append(("poi-%d" % k, r, 5.0, 0.0))
        edges.append((r, "poi-%d" % k, float(rng.uniform(1, 100)), 0.0))
        edges.append(("poi-%d" % k, "poi-%d" % k, 1.0, 0.0))
    order = rng.permutation(len(edges))
    return graphml_doc(nodes, [edges[i] for i in order], directed=True)


def test_one_way_region_topology_rejected():
    """Without the two arcs back the side regions are one-way: not strongly connected, which the
    reference refuses at load (critical + NULL, shd-topology.c:134-151) -- so sources that cannot
    reach the landmark, or targets the landmark cannot reach, never reach the kernels."""
    top = sa.Topology.from_buffer(_one_way_regions_graphml(with_back=False))
    assert top is None or not getattr(top, "_h", None)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["batch", "replay_all"])
def test_directed_near_one_way_regions(mode):
    """a directed fixture with near one-way regions -- a sink region left and a source
    region entered only through one 5,000 ms arc each -- so d(v, h0) (potSrc) and d(h0, v)
    (kappa) are huge for one side each, and the two directions of most pairs differ by orders of
    magnitude.  Batch mode (flagged rows through the replay) and replay_all against the oracle,
    bit for bit, with no error and no -1 pair."""
    data = _one_way_regions_graphml()
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    assert top.is_directed and not top.is_complete
    if mode == "replay_all":
        top.set_option("replay_all", 1)
    else:
        top.set_option("tie_dense", 0)
    otop, ips, verts = attach_hosts(top, g, 90, geo_hints=None)
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert st["errors"] == 0 and np.all(lat > 0) and np.all(rel > 0)
    assert lat.max() > 5000.0 and lat.min() < 100.0  # the long arcs are on some paths
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
