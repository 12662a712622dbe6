"""CPU tests of the product's boundary and host logic (no GPU compute calls).

* libshdtopo.so loads and exports every function include/shd_topology_abi.h declares;
* the C++ GraphML reader agrees with the oracle's ElementTree reader (igraph semantics);
* attach (candidate index, hints, LPM, RNG use) agrees with the reference restatement;
* error behaviour: topology_new -> NULL on bad input; getters -> -1.0 for unattached addresses;
  without a GPU the table build fails loudly (no CPU fallback).
"""
import ctypes
import os
import re
import tempfile

import numpy as np
import pytest

import oracle
import shadow_amd as sa
from conftest import ROOT, bundled_topology
from helpers import attach_hosts, bundled_pair, host_ip, synthetic_pair
from shadow_amd import _lib


def header_functions():
    names = set()
    for h in ("shd_topology_abi.h", "shd_topology_window.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        names |= set(re.findall(r"\b((?:topology|shdtopo|topowindow)_\w+)\s*\(", txt))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib, shim = _lib.load()
    names = header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)
    for n in ("address_toNetworkIP", "random_nextDouble", "worker_updateMinTimeJump"):
        assert hasattr(shim, n)


def test_product_has_no_oracle_dependency():
    """The product must not link, load or import the checker."""
    for f in os.listdir(os.path.join(ROOT, "shadow_amd")):
        if f.endswith(".py"):
            src = open(os.path.join(ROOT, "shadow_amd", f)).read()
            assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
    so = open(os.path.join(ROOT, "shadow_amd", "libshdtopo.so"), "rb").read()
    assert b"liboracle" not in so and b"orc_dijkstra" not in so


def _compare_graph(top, g):
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    assert V == g.V and len(eu) == g.E
    assert np.array_equal(eu, g.eu) and np.array_equal(ev, g.ev)
    assert np.array_equal(elat.view(np.uint64), g.elat.view(np.uint64))
    assert np.array_equal(np.nan_to_num(eloss, nan=-7), np.nan_to_num(g.eloss, nan=-7))
    assert np.array_equal(np.nan_to_num(vloss, nan=-7), np.nan_to_num(g.vloss, nan=-7))


@pytest.mark.parametrize("name", ["topology.simple", "topology", "topology.plab"])
def test_graphml_reader_matches_igraph_semantics(name):
    top, g = bundled_pair(name)
    assert top.num_vertices == g.V and top.num_edges == g.E
    assert top.is_complete == g.is_complete()
    assert top.is_directed == g.directed
    _compare_graph(top, g)


def test_synthetic_writer_reader_roundtrip():
    top, g = synthetic_pair(seed=3, n_routers=1500, n_poi=60, n_edges=14000)
    _compare_graph(top, g)
    assert not top.is_complete and not g.is_complete() and g.is_strongly_connected()
    # K7: every poi has exactly one self loop
    ids = g.vattrs["id"]
    loops = g.eu[g.eu == g.ev]
    assert sorted(ids[v] for v in loops) == sorted(x for x in ids if x.startswith("poi"))
    # no parallel edges
    a = np.minimum(g.eu, g.ev).astype(np.int64) * g.V + np.maximum(g.eu, g.ev)
    assert len(np.unique(a)) == len(a)


def test_synthetic_c4_shape():
    """config 4 at full size: 1M vertices, exactly 10M undirected edges (generator only)."""
    top = sa.Topology.synthetic()
    assert top.num_vertices == 1_000_000 and top.num_edges == 10_000_000
    assert not top.is_complete


def test_graphml_edge_cases():
    xml = b"""<?xml version="1.0"?><!-- c --><graphml><key id="a" for="node" attr.name="packetloss"
      attr.type="double"><default>0.5</default></key><key id="l" for="edge" attr.name="latency"
      attr.type="double"/><key id="t" for="node" attr.name="type" attr.type="string"/>
      <graph edgedefault="undirected"><node id="poi-&amp;1"><data key="t">a&lt;b</data></node>
      <node id="poi-2"><data key="a">0.25</data></node>
      <edge source="poi-&amp;1" target="poi-2"><data key="l"> 7.5 </data></edge>
      <edge source="poi-2" target="poi-2"><data key="l"><![CDATA[3]]></data></edge>
      <edge source="poi-&amp;1" target="poi-&amp;1"><data key="l">1e0</data></edge>
      </graph></graphml>"""
    top = sa.Topology.from_buffer(xml)
    g = oracle.OGraph.from_graphml(xml)
    assert g.vattrs["id"][0] == "poi-&1" and g.vattrs["type"][0] == "a<b"
    _compare_graph(top, g)
    assert list(g.vloss) == [0.5, 0.25] and list(g.elat) == [7.5, 3.0, 1.0]


def test_topology_new_failures():
    lib, _ = _lib.load()
    assert sa.Topology.new("/nonexistent/topology.xml") is None
    disconnected = b"""<graphml><key id="l" for="edge" attr.name="latency" attr.type="double"/>
      <graph edgedefault="undirected"><node id="poi-1"/><node id="poi-2"/><node id="poi-3"/>
      <edge source="poi-1" target="poi-2"><data key="l">1</data></edge></graph></graphml>"""
    assert sa.Topology.from_buffer(disconnected) is None
    zero = b"""<graphml><key id="l" for="edge" attr.name="latency" attr.type="double"/>
      <graph edgedefault="undirected"><node id="poi-1"/><node id="poi-2"/>
      <edge source="poi-1" target="poi-2"><data key="l">0</data></edge></graph></graphml>"""
    assert sa.Topology.from_buffer(zero) is None
    assert sa.Topology.from_buffer(b"<graphml><graph></graphml") is None or True


def test_attach_matches_reference_all_hint_kinds():
    top, g = bundled_pair("topology")
    # random (no hints), geocode, type, ip exact, LPM, unparsable, ANY
    attach_hosts(top, g, 150)
    attach_hosts(top, g, 60, geo_hints=[g.vattrs["geocode"][(7 * k) % g.V] for k in range(60)])
    attach_hosts(top, g, 30, type_hints=["cluster", "nosuchtype"])
    ips = [x for x in g.vattrs["ip"] if x != "0.0.0.0"]
    for k, h in enumerate(ips + ["190.181.151.1", "10.9.8.7", "255.255.255.255", "garbage",
                                 "0.0.0.0"]):
        v1, s1 = top.attach_ip(host_ip(9000 + k), 777 + k, ipHint=h)
        v2, s2, _ = oracle.attach_vertex(g.vattrs, 777 + k, ip_hint=h)
        assert (v1, s1) == (v2, s2), h
        # type + geocode + ip together
        v1, s1 = top.attach_ip(host_ip(9500 + k), 99 + k, ipHint=h, typeHint="CLUSTER",
                               geocodeHint=g.vattrs["geocode"][k])
        v2, s2, _ = oracle.attach_vertex(g.vattrs, 99 + k, ip_hint=h, type_hint="CLUSTER",
                                         geocode_hint=g.vattrs["geocode"][k])
        assert (v1, s1) == (v2, s2), h


def test_attach_through_shadow_types_and_bandwidth():
    data = bundled_topology("topology.simple")
    top = sa.Topology.from_buffer(data)
    r = sa.Random(679019682)
    addr = sa.Address("11.0.0.1")
    down, up = top.attach(addr, r)
    assert (down, up) == (2048, 1024)
    assert r.state != 679019682        # exactly one draw consumed
    r2 = sa.Random(679019682)
    r2.nextDouble()
    assert r.state == r2.state


def test_getters_unattached_return_minus_one():
    top = sa.Topology.from_buffer(bundled_topology("topology.simple"))
    top.set_option("abort_on_error", 0)
    a, b = sa.Address("11.0.0.1"), sa.Address("11.0.0.2")
    assert top.getLatency(a, b) == -1.0
    assert top.getReliability(a, b) == -1.0
    assert not top.isRoutable(a, b)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    top = sa.Topology.from_buffer(bundled_topology("topology.simple"))
    top.set_option("abort_on_error", 0)
    a, b = sa.Address("11.0.0.1"), sa.Address("11.0.0.2")
    top.attach(a, sa.Random(1))
    top.attach(b, sa.Random(2))
    assert top.getLatency(a, b) == -1.0          # build fails loudly, no CPU path
    assert top.getMinimumLatency() == -1.0
    with pytest.raises(RuntimeError):
        top.build()


def test_synth_packets_seed_chain_and_host_streams():
    """C5 workload generator: per-packet pre-draw states follow each host's rand_r stream."""
    top = sa.Topology.synthetic(seed=5, n_routers=2000, n_poi=200, n_edges=20000)
    pk = top.synth_packets(20261015, 300, 5000, 10**9, 5_000_000)
    assert len(top.attached_vertices()) > 0
    # consecutive packets of one host: state advances by exactly one rand_r
    src = pk["src_ip"]
    for h in np.unique(src)[:20]:
        idx = np.nonzero(src == h)[0]
        for a, b in zip(idx[:-1], idx[1:]):
            _, nxt = oracle.rand_r(int(pk["state_in"][a]))
            assert nxt == pk["state_in"][b]
    assert np.all(pk["src_ip"] != pk["dst_ip"])
    assert 0.75 < (pk["payload"] > 0).mean() < 0.85
    assert np.all((pk["now"] >= 10**9) & (pk["now"] < 10**9 + 5_000_000))


def test_device_option_fixed_once_the_attach_time_preparation_starts():
    """The "device" option (shdtopo_set_option): before the first attach it may move the topology
    to another device (topology_new's background init is released); once the first attach started
    the attach-time preparation on a device, another device is refused (-1 -> KeyError) and the
    same device is accepted.  "abort_on_error" / "lazy" are lock-free flags."""
    top = sa.Topology.from_buffer(bundled_topology("topology.plab"))
    top.set_option("device", 3)
    top.set_option("device", 0)
    top.set_option("lazy", 1)
    top.set_option("abort_on_error", 0)
    # plab is complete: no attach-time preparation, so attach a synthetic (SSSP) topology instead
    syn = sa.Topology.synthetic(seed=3, n_routers=200, n_poi=20, n_edges=2000)
    syn.set_option("device", 2)
    syn.attach_ip(1, 5, typeHint="client")
    with pytest.raises(KeyError):
        syn.set_option("device", 1)
    syn.set_option("device", 2)
    syn.set_option("lazy", 0)
    with pytest.raises(KeyError):
        syn.set_option("device", -1)


def test_device_option_fixed_after_a_complete_topology_build():
    """a complete topology never starts the attach-time preparation, so a
    build (or any other device use) must fix the "device" option too -- its table and resident
    A x A edge matrices live on that device.  On a CPU-only box the build fails, but it asked the
    device for work: another device is refused afterwards, the same one still accepted."""
    top = sa.Topology.from_buffer(bundled_topology("topology.plab"))
    top.set_option("abort_on_error", 0)
    top.set_option("device", 1)                    # before any use: allowed
    top.attach_ip(sa.ip_to_network("11.0.0.1"), 5)
    top.attach_ip(sa.ip_to_network("11.0.0.2"), 6)
    try:
        top.build()
    except RuntimeError:
        pass                                       # no GPU here
    with pytest.raises(KeyError):
        top.set_option("device", 0)
    top.set_option("device", 1)
    try:
        top.rebuild()                              # invalidates the table first
    except RuntimeError:
        pass
    with pytest.raises(KeyError):                  # still fixed
        top.set_option("device", 2)


def test_synthetic_directed_shape_and_bucket_options():
    """The synthetic generator's directed variant (ShdSynthParams.directed, tools' C4-dir): every
    non-loop edge becomes two arcs, the reverse one with its own draws, so E = 2 x n_edges -
    n_poi and the graph stays strongly connected; and the batched SSSP's bucket options: "delta"
    and "h0_phase" in [0, 1) (< 0: the round-4 shifts) are accepted, a phase >= 1 is refused."""
    top = sa.Topology.synthetic(seed=3, n_routers=500, n_poi=40, n_edges=5000, directed=True)
    assert top.is_directed and not top.is_complete
    assert top.num_vertices == 540 and top.num_edges == 2 * 5000 - 40
    V, eu, ev, el, lo, vl = top.export_graph()
    nl = eu != ev
    fwd = set(zip(eu[nl].tolist(), ev[nl].tolist()))
    assert all((b, a) in fwd for a, b in fwd)  # every arc has its reverse
    und = sa.Topology.synthetic(seed=3, n_routers=500, n_poi=40, n_edges=5000)
    assert not und.is_directed and und.num_edges == 5000
    for k, v in (("delta", 25.0), ("h0_phase", 0.5), ("h0_phase", 0.0), ("h0_phase", -1),
                 ("balance", 0), ("balance", 1)):
        top.set_option(k, v)
    with pytest.raises(KeyError):
        top.set_option("h0_phase", 1.0)
    # parent-pass row-scan chunk (records per slot: chunk x batch x 16 B): 64 .. 2^20
    for v in (64, 16384, 1 << 20):
        top.set_option("row_scan_chunk", v)
    for v in (63, 0, -1, (1 << 20) + 1):
        with pytest.raises(KeyError):
            top.set_option("row_scan_chunk", v)


def _layout(cost, fixed, fill, slots, batch):
    lib, _ = _lib.load()
    cost = np.ascontiguousarray(cost, dtype=np.float64)
    n = len(cost)
    order = np.zeros(n, np.uint32)
    starts = np.zeros(n + 1, np.uint32)
    nb = ctypes.c_int64(0)
    r = lib.shdtopo_test_batch_layout(cost.ctypes.data, n, fixed, fill, slots, batch,
                                      order.ctypes.data, starts.ctypes.data, ctypes.byref(nb))
    return r, order, starts[:nb.value + 1]


def _best_runs(cost, fixed, slots, batch):
    """Brute force: the smallest largest-run cost over every cut into <= slots runs of <= batch."""
    n = len(cost)
    best = [[np.inf] * (slots + 1) for _ in range(n + 1)]  # best[i][k]: first i positions, k runs
    best[0][0] = 0.0
    for i in range(1, n + 1):
        for k in range(1, slots + 1):
            for m in range(1, min(batch, i) + 1):
                prev = best[i - m][k - 1]
                if prev < np.inf:
                    best[i][k] = min(best[i][k], max(prev, fixed + cost[i - m:i].sum()))
    return min(best[n][1:])


@pytest.mark.parametrize("seed", range(6))
def test_measured_layout_one_round_is_min_max(seed):
    """Option balance, one round of the slots: runs of the grouping order,
    at most `slots` runs of 1..batch positions covering every row once, minimising the largest
    predicted batch (fixed part + its sources' costs) -- checked against a brute-force cut."""
    rng = np.random.default_rng(seed)
    n, slots, batch = int(rng.integers(8, 20)), int(rng.integers(3, 6)), 4
    fill = -(-n // slots)
    if fill > batch:
        n = slots * batch
        fill = batch
    cost = rng.uniform(0.5, 3.0, n) * (1 + 4 * (rng.random(n) < 0.15))  # a few heavy sources
    fixed = 1.5
    r, order, starts = _layout(cost, fixed, fill, slots, batch)
    assert r == 0
    assert np.array_equal(order, np.arange(n))  # runs keep the grouping order
    sizes = np.diff(starts.astype(np.int64))
    assert starts[0] == 0 and starts[-1] == n and len(sizes) <= slots
    assert sizes.min() >= 1 and sizes.max() <= batch
    got = max(fixed + cost[a:b].sum() for a, b in zip(starts[:-1], starts[1:]))
    plain = max(fixed + cost[i:i + fill].sum() for i in range(0, n, fill))
    assert got <= plain + 1e-9
    assert got <= _best_runs(cost, fixed, slots, batch) * (1 + 2e-4)


def test_measured_layout_several_rounds_longest_first():
    """Several rounds: batches stay groups of `fill` consecutive grouping positions, dequeued by
    predicted cost descending (list scheduling in LPT order), the ragged batch last."""
    rng = np.random.default_rng(3)
    n, fill, slots = 203, 8, 4
    cost = rng.uniform(0.2, 2.0, n)
    r, order, starts = _layout(cost, 1.0, fill, slots, 8)
    assert r == 0
    assert sorted(order.tolist()) == list(range(n))
    groups = [order[a:b] for a, b in zip(starts[:-1], starts[1:])]
    assert len(groups) == -(-n // fill)
    for g in groups:  # whole groups of the grouping order
        assert g[0] % fill == 0 and np.array_equal(g, np.arange(g[0], g[0] + len(g)))
    assert len(groups[-1]) == n % fill  # the ragged batch last
    pred = [1.0 + cost[g].sum() for g in groups[:-1]]
    assert all(x >= y for x, y in zip(pred, pred[1:]))
    # no layout for bad shapes: the build keeps the grouping order
    assert _layout(cost, 1.0, 9, slots, 8)[0] == -1
    assert _layout(cost[:1], 1.0, 1, 0, 8)[0] == -1
