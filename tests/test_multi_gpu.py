"""Multi-GPU build inside libshdtopo (option "devices"): one Shadow process, no
Python in the loop -- rows sharded over devices, RCCL all-gather of the rows and all-reduce(MIN)
of the runahead minimum.

CPU: the row split (shdtopo_shard_rows) for N = 1, 2, 3, 8 covers every row exactly once and
agrees with the multi-process harness (shadow_amd.sharding).  GPU (one MI355X on the test box):
the RCCL exchange with one device, and 2 / 3 engines on the same device (RCCL refuses duplicate
devices, so those exchange by device copies), each bit-equal to the single-device table and to
the oracle.
"""
import ctypes

import numpy as np
import pytest

import oracle
import shadow_amd as sa
from shadow_amd import sharding
from helpers import attach_hosts, random_topology_graphml, synthetic_pair


@pytest.mark.parametrize("n", [1, 2, 3, 8])
@pytest.mark.parametrize("A", [1, 7, 37, 10000])
def test_shard_rows_cover_each_row_once(n, A):
    lib, _ = sa._lib.load()
    seen = np.zeros(A, np.int32)
    prev = 0
    for d in range(n):
        r0, r1 = ctypes.c_int64(), ctypes.c_int64()
        lib.shdtopo_shard_rows(A, n, d, ctypes.byref(r0), ctypes.byref(r1))
        assert r0.value == prev and r0.value <= r1.value
        assert (r1.value - r0.value) <= -(-A // n)
        assert (r0.value, r1.value) == sharding.shard_range(A, d, n)
        seen[r0.value:r1.value] += 1
        prev = r1.value
    assert prev == A and np.all(seen == 1)


def _table_with(devices, rccl, integer, seed=21):
    top, g = synthetic_pair(seed=seed, n_routers=2000, n_poi=101, n_edges=20000, integer=integer)
    top.set_option("devices", devices)
    top.set_option("rccl", int(rccl))
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    return top, g, otop, ips, verts, a, lat, rel, hops


@pytest.mark.gpu
@pytest.mark.parametrize("integer", [False, True])
@pytest.mark.parametrize("devices,rccl", [(1, True), (2, False), (3, False)])
def test_multi_device_table_equals_single_and_oracle(devices, rccl, integer):
    top1, g, _, _, verts, a1, lat1, rel1, hops1 = _table_with(1, False, integer)
    topN, _, otop, ips, _, aN, latN, relN, hopsN = _table_with(devices, rccl, integer)
    st = topN.stats()
    assert st["devices"] == devices and st["errors"] == 0
    if rccl:
        assert st["exchange_ms"] > 0
    assert np.array_equal(a1, aN)
    assert np.array_equal(lat1.view(np.uint64), latN.view(np.uint64))
    assert np.array_equal(rel1.view(np.uint64), relN.view(np.uint64))
    assert np.array_equal(hops1, hopsN)
    assert topN.getMinimumLatency() == top1.getMinimumLatency()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(latN.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(relN.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hopsN, ohops.astype(np.uint16))
    assert topN.getMinimumLatency() == olat.min()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [2, 3])
def test_directed_multi_device_table_equals_oracle(devices):
    """A directed topology on devices = N engines: the peers copy the owner's out-rows and in-rows
    (d_adjo, d_rowptrIn) with the rest of the prepared graph; every pair bit-exact against the
    oracle."""
    data = random_topology_graphml(n_routers=4000, n_poi=60, extra=20000, seed=13, directed=True)
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    top.set_option("devices", devices)
    top.set_option("rccl", 0)
    otop, ips, verts = attach_hosts(top, g, 150, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    assert st["devices"] == devices and st["errors"] == 0 and st["replay_rows"] == 0
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert top.getMinimumLatency() == olat.min()


@pytest.mark.gpu
def test_getters_trigger_multi_device_build():
    """topology_getLatency on a topology with devices = 2: the lazy getter builds the table on
    both engines itself (no Python sharding) and answers as the reference cache does."""
    top, g = synthetic_pair(seed=23, n_routers=1500, n_poi=70, n_edges=15000, integer=True)
    top.set_option("devices", 2)
    otop, ips, verts = attach_hosts(top, g, 150, type_hints=["client", "relay"])
    rng = np.random.default_rng(4)
    for _ in range(300):
        x, y = (int(v) for v in rng.choice(ips, 2))
        assert top.latency_ip(x, y) == otop.get_latency(x, y)
        assert top.reliability_ip(x, y) == otop.get_reliability(x, y)
    assert top.stats()["devices"] == 2
    assert top.lazyMinimumLatency() == otop.minimum_path_latency


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [2, 3])
def test_multi_device_build_prepares_the_graph_once(devices):
    """One multi-GPU build prepares the graph once (on the owner's device) and the peer engines
    copy its device CSR and share its host arrays: one host preparation per build, none in the
    next build, and the peers' tables equal the owner's (checked against the oracle above)."""
    top, g = synthetic_pair(seed=37, n_routers=2500, n_poi=120, n_edges=25000)
    top.set_option("devices", devices)
    top.set_option("prepare_on_attach", 0)  # the build itself prepares the graph (counted below)
    otop, ips, verts = attach_hosts(top, g, 200, type_hints=["client", "relay"])
    top.build()
    st = top.stats()
    assert st["devices"] == devices and st["csr_host_runs"] == 1 and st["csr_ms"] > 0
    assert st["exchange_kind"] == 2  # engines sharing the test box's one device: push copies
    top.rebuild()
    st = top.stats()
    assert st["csr_host_runs"] == 0 and st["csr_ms"] == 0
    a, lat, rel, hops = top.table()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.gpu
def test_route_on_every_device_slot():
    """shdtopo_route_batch_device_slot: every engine of a devices = 3 Topology holds the whole
    table after the exchange and routes a window slice bit-exactly like slot 0."""
    import torch
    top, g = synthetic_pair(seed=39, n_routers=1500, n_poi=80, n_edges=15000)
    top.set_option("devices", 3)
    attach_hosts(top, g, 150, type_hints=["client", "relay"])
    a, lat, rel, hops = top.table()
    A, n = len(a), 5000
    rng = np.random.default_rng(9)
    s = rng.integers(0, A, n).astype(np.int32)
    d = rng.integers(0, A, n).astype(np.int32)
    pay = np.where(rng.random(n) < 0.8, 1448, 0).astype(np.int32)
    sin = rng.integers(0, 2**31, n).astype(np.int32)
    now = rng.integers(10**9, 2 * 10**9, n).astype(np.int64)
    cu = lambda x: torch.from_numpy(x).cuda()
    outs = []
    for slot in range(3):
        t_out = torch.empty(n, dtype=torch.int64, device="cuda")
        s_out = torch.empty(n, dtype=torch.int32, device="cuda")
        d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
        top.route_batch_device_slot(slot, cu(s), cu(d), cu(pay), cu(sin), cu(now), 4_000_000, 1,
                                    t_out, s_out, d_out)
        torch.cuda.synchronize()
        outs.append((t_out.cpu().numpy(), s_out.cpu().numpy(), d_out.cpu().numpy()))
    ot, od, os_ = oracle.route_packets(lat[s, d], rel[s, d], pay.view(np.uint32),
                                       sin.view(np.uint32), now.view(np.uint64), 4_000_000, 1)
    for t_, s_, d_ in outs:
        assert np.array_equal(t_.view(np.uint64), ot)
        assert np.array_equal(s_.view(np.uint32), os_)
        assert np.array_equal(d_, od)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [2, 3])
def test_multi_device_default_attach_prep_prepares_once(devices):
    """The default path of a Shadow run (prepare_on_attach left on): the first attach starts the
    attach-time preparation thread on the owner's device, and the devices = N build that follows
    copies its graph to the peer engines -- one host preparation in all (attach-time thread +
    builds, owner + peers), none in a rebuild, and every engine's table equals the oracle's."""
    top, g = synthetic_pair(seed=41, n_routers=2500, n_poi=120, n_edges=25000)
    top.set_option("devices", devices)
    otop, ips, verts = attach_hosts(top, g, 200, type_hints=["client", "relay"])
    top.build()
    st = top.stats()
    assert st["devices"] == devices and st["errors"] == 0
    # by the attach-time thread (csr_host_runs 0), or by the build if it took the lock first
    assert st["csr_host_runs_total"] == 1 and st["csr_host_runs"] in (0, 1)
    top.rebuild()
    st = top.stats()
    assert st["csr_host_runs_total"] == 1 and st["csr_host_runs"] == 0
    a, lat, rel, hops = top.table()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert top.getMinimumLatency() == olat.min()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["topology", "topology.plab"])
@pytest.mark.parametrize("devices", [8])
def test_complete_branch_devices8_equals_oracle(name, devices):
    """BASELINE config 3 ("all-pairs table on 8 MI355X") through the library's multi-device build:
    the complete branch's rows sharded over 8 engines (C3: 183 rows -> 23 per engine, the last one
    short), each engine's pair_table_complete_kernel, the row exchange and the all-reduce of the
    minimum (device copies: the test box's engines share one GPU).  One host per vertex by its
    unique geocode; every pair bit-exact against _topology_lookupPath's
    restatement, the runahead minimum too (shd-master.c:113-124 consumes it)."""
    from helpers import bundled_pair
    top, g = bundled_pair(name)
    assert top.is_complete
    top.set_option("devices", devices)
    geos = list(g.vattrs["geocode"])
    assert len(set(geos)) == len(geos)
    otop, ips, verts = attach_hosts(top, g, g.V, geo_hints=geos)
    a, lat, rel, hops = top.table()
    st = top.stats()
    A = len(a)
    assert st["devices"] == devices and st["errors"] == 0 and A == g.V
    R = -(-A // devices)
    assert st["device_rows"][:devices] == [max(0, min(A, (d + 1) * R) - min(A, d * R))
                                           for d in range(devices)]
    assert all(st["device_kernel_ms"][d] > 0 for d in range(devices) if st["device_rows"][d])
    assert st["exchange_bytes"] == (devices - 1) * R * (A * 18 + 8)
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.all(hops == 1)
    assert top.getMinimumLatency() == olat.min()
    # a rebuild reuses the resident edge matrices of every engine (same attached set)
    nb = st["pair_matrix_builds"]
    top.rebuild()
    assert top.stats()["pair_matrix_builds"] == nb
    a2, lat2, rel2, _ = top.table()
    assert np.array_equal(lat2.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel2.view(np.uint64), orel.view(np.uint64))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_full_size_c4_devices8_equals_devices1():
    """BASELINE config 4 at full size (1M vertices / 10M edges, 10,000 x
    10,000 table) built by 8 engines -- rows sharded over them, each shard pushed into the other
    engines' tables as soon as it is done (exchange_kind 2; on the one-GPU test box the engines
    share the device, so RCCL is not possible and the push is the exchange).  The table
    must equal the devices = 1 table bit for bit (latency, reliability and hops hashed),
    getMinimumLatency must be equal (the all-reduced minimum, shd-master.c:113-124), and 16 seeded
    rows must equal the oracle's Dijkstra + helper."""
    import hashlib
    import os
    top = sa.Topology.synthetic(seed=20261015)
    top.synth_packets(20261015, 100_000, 0, 10**9, 10**7)
    att = top.attached_vertices()
    A = len(att)
    top.set_option("devices", 8)
    a8, lat8, rel8, hop8 = top.table()
    st = top.stats()
    assert st["devices"] == 8 and st["exchange_kind"] == 2 and st["errors"] == 0
    assert sum(st["device_rows"]) == A and st["exchange_exposed_ms"] <= st["exchange_ms"]
    m8 = top.getMinimumLatency()
    digest = lambda *xs: hashlib.sha256(b"".join(x.tobytes() for x in xs)).hexdigest()
    h8 = digest(lat8, rel8, hop8)
    rows = np.sort(np.random.default_rng(8).choice(A, 16, replace=False))
    sl, sr, sh = lat8[rows].copy(), rel8[rows].copy(), hop8[rows].copy()
    del lat8, rel8, hop8
    top.set_option("devices", 1)
    a1, lat1, rel1, hop1 = top.table()
    assert top.stats()["devices"] == 1
    assert np.array_equal(a1, a8)
    assert digest(lat1, rel1, hop1) == h8
    assert top.getMinimumLatency() == m8 == float(lat1.min())
    del lat1, rel1, hop1
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    g = oracle.OGraph(V, eu, ev, elat, eloss, vloss)
    olat, orel, ohops = g.source_rows(att[rows], att, nthreads=min(16, os.cpu_count() or 1))
    assert np.array_equal(sl.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(sr.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(sh, ohops.astype(np.uint16))
