"""GPU parity: the HIP path (libshdtopo.so) against the CPU oracle on the same inputs.

Bit-exact for latency, hops and the packet route (integer/byte/time outputs); reliability is
checked bit-exact as well (the kernels multiply in the reference order) and, as the north star
states, at worst within 1e-12 relative.
"""
import numpy as np
import pytest

import oracle
import shadow_amd as sa
from helpers import attach_hosts, bundled_pair, host_ip, rel_close, scipy_rows, synthetic_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["topology.simple", "topology", "topology.plab"])
def test_complete_table_bundled(name):
    """configs 1-3: every attached pair through pair_table_complete vs _topology_lookupPath."""
    top, g = bundled_pair(name)
    assert top.is_complete and g.is_complete()
    geos = list(g.vattrs["geocode"])
    # one host per vertex where geocodes are unique (plab, full); simple: random attach
    hints = geos if len(set(geos)) == len(geos) else None
    n = g.V if hints else 2
    otop, ips, verts = attach_hosts(top, g, n, geo_hints=hints)
    a, lat, rel, hops = top.table()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.all(hops == 1)
    assert top.getMinimumLatency() == olat.min()


@pytest.mark.parametrize("fill", [1, 8])
@pytest.mark.parametrize("hubs", [-1, 0, 700])
@pytest.mark.parametrize("integer", [False, True])
def test_sssp_synthetic_table(integer, hubs, fill):
    """SSSP branch: sssp_batch_kernel (8 sources per workgroup; fill 1 = one source per batch),
    plus the heap replay of tie rows, vs the igraph-0.7 Dijkstra + helper restatement.  `hubs`
    caps the LDS-resident distance rows: all (-1: as many as fit), none, or mixed."""
    top, g = synthetic_pair(seed=11, n_routers=3000, n_poi=150, n_edges=30000, integer=integer)
    top.set_option("lds_hubs", hubs)
    top.set_option("batch_fill", fill)  # whole batches (auto would run 1 source per slot here)
    top.set_option("tie_dense", 0)  # the batch kernel + flagged-row replay path (no tie probe)
    otop, ips, verts = attach_hosts(top, g, 400, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert st["errors"] == 0
    # latency == dist: bit-exact on every pair, ties or not
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    # every pair bit-exact, integer ties included: the batch kernel flags the rows whose target
    # chains cross a d-tied parent and the heap replay recomputes them in igraph's pop order
    if integer:
        assert st["ambiguous_pairs"] > 0 and st["replay_rows"] > 0
    else:
        assert st["ambiguous_pairs"] == 0 and st["replay_rows"] == 0
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert top.getMinimumLatency() == olat.min()


@pytest.mark.parametrize("integer", [False, True])
def test_target_skip_exact_across_target_sets(integer):
    """The batch relaxation drops pairs into non-target tail vertices that would expand nothing
    (target bits in the relaxation copy).  Tables with the skip on equal the oracle and the
    skip-off tables bit for bit, before and after a late attach changes the target set (the
    bits are re-marked)."""
    tops = []
    for skip in (1, 0):
        top, g = synthetic_pair(seed=17, n_routers=3000, n_poi=150, n_edges=30000, integer=integer)
        top.set_option("target_skip", skip)
        top.set_option("batch_fill", 8)
        top.set_option("tie_dense", 0)  # the batch kernel path (no tie probe)
        tops.append(top)
    verts = []
    st = 1
    for lo, hi in ((0, 120), (120, 300)):  # second round: a late attach of new hosts
        for k in range(lo, hi):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            th = ("client", "relay")[k % 2]
            got = {top.attach_ip(host_ip(k + 1), st, typeHint=th) for top in tops}
            assert len(got) == 1
            verts.append(got.pop()[0])
        oa, olat, orel, ohops = g.table(verts)
        for top in tops:
            a, lat, rel, hops = top.table()
            assert np.array_equal(a, oa)
            assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
            assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
            assert np.array_equal(hops, ohops.astype(np.uint16))
        assert len(oa) > 0


@pytest.mark.parametrize("integer", [False, True])
def test_single_slot_reuses_touched_lines(integer):
    """One SSSP slot runs every batch: each batch resets only the distance lines the previous
    batches of the slot lowered from +inf (the touched-line bitmap), never the whole [V][K]
    block.  Two builds (the second after a late attach) equal the oracle bit for bit."""
    top, g = synthetic_pair(seed=23, n_routers=3000, n_poi=150, n_edges=30000, integer=integer)
    top.set_option("slots", 1)
    top.set_option("batch_fill", 3)
    top.set_option("tie_dense", 0)  # the batch kernel path (no tie probe)
    verts = []
    st = 7
    for lo, hi in ((0, 90), (90, 260)):
        for k in range(lo, hi):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            v, _ = top.attach_ip(host_ip(k + 1), st, typeHint=("client", "relay")[k % 2])
            verts.append(v)
        a, lat, rel, hops = top.table()
        s_ = top.stats()
        assert s_["slots"] == 1 and s_["errors"] == 0
        assert 0 < s_["touched_lines"] < len(a) * top.num_vertices
        oa, olat, orel, ohops = g.table(verts)
        assert np.array_equal(a, oa)
        assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
        assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
        assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("toggle", ["target_skip", "target_resort"])
def test_target_options_toggled_on_one_topology(toggle):
    """the target-aware re-sort rewrites the relaxation copy for one target set.
    Turning the skip (or the re-sort) off on the same Topology and then changing the target set
    must not leave the old set's keys in the copy: it is restored from the plain adjacency."""
    top, g = synthetic_pair(seed=29, n_routers=3000, n_poi=150, n_edges=30000)
    top.set_option("batch_fill", 8)
    verts = []
    st = 3
    for rnd, (lo, hi) in enumerate(((0, 100), (100, 240), (240, 330))):
        for k in range(lo, hi):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            v, _ = top.attach_ip(host_ip(k + 1), st, typeHint=("client", "relay")[k % 2])
            verts.append(v)
        a, lat, rel, hops = top.table()
        oa, olat, orel, ohops = g.table(verts)
        assert np.array_equal(a, oa)
        assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
        assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
        assert np.array_equal(hops, ohops.astype(np.uint16))
        top.set_option(toggle, rnd % 2)  # off after round 0, on again after round 1


def test_iteration_guard_error_then_clean_build():
    """The batch kernel's iteration guard (a batch that never settles) is reported: the build
    returns -4 (abort() under the default abort_on_error), and the next build with the guard
    restored is bit-exact -- nothing of the aborted batches leaks into it."""
    top, g = synthetic_pair(seed=31, n_routers=2000, n_poi=101, n_edges=20000)
    top.set_option("abort_on_error", 0)
    otop, ips, verts = attach_hosts(top, g, 250, type_hints=["client", "relay"])
    top.set_option("iter_guard", 3)
    with pytest.raises(RuntimeError, match="-4"):
        top.build()
    top.set_option("iter_guard", 4e6)
    a, lat, rel, hops = top.table()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("batch", [2, 4, 16])
def test_sssp_batch_widths(batch):
    """Every batch width settles the same table (ragged last batch included: A % K != 0)."""
    top, g = synthetic_pair(seed=17, n_routers=2000, n_poi=101, n_edges=20000)
    top.set_option("batch", batch)
    top.set_option("batch_fill", batch)
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert len(a) % batch != 0 or batch == 2
    assert st["errors"] == 0 and st["ambiguous_pairs"] == 0
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("fill", [0, 1, 3, 5, 8])
@pytest.mark.parametrize("integer", [False, True])
def test_sssp_batch_fill(fill, integer):
    """Batches filled below K (option batch_fill; 0 = auto, which fills ceil(A / slots) here:
    a slot per source for this short table) settle the same table: idle lanes, the ragged last
    batch and the batch order by mean pi."""
    top, g = synthetic_pair(seed=19, n_routers=2000, n_poi=101, n_edges=20000, integer=integer)
    top.set_option("batch_fill", fill)
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    assert st["errors"] == 0
    assert st["batch_fill"] == (fill if fill else min(8, -(-len(a) // st["slots"])))
    if fill == 0:  # a fresh workspace gets a slot per source (up to the CUs), not per batch of K
        import torch
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        assert st["slots"] == min(len(a), cus)
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("order,slots,fill", [(2, 8, 0), (4, 8, 0), (5, 8, 0), (5, 64, 0),
                                              (3, 8, 5), (1, 8, 2)])
def test_sssp_batch_order_and_rounds(order, slots, fill):
    """The batch dequeue order (batch_order 1 shuffled, 2 / 3 mean pi, 4 h0-tree depth, 5 auto:
    depth past 3 rounds of the slots) and the auto fill by equal rounds on few slots (many
    rounds, ragged last batches) settle the same table, bit-exact against the oracle."""
    top, g = synthetic_pair(seed=23, n_routers=2000, n_poi=101, n_edges=20000)
    top.set_option("batch_order", order)
    top.set_option("slots", slots)
    top.set_option("batch_fill", fill)
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    assert st["errors"] == 0
    if fill == 0:  # equal rounds: the fewest sources per batch that keep the round count
        S = st["slots"]
        rounds = -(-len(a) // (8 * S))
        assert st["batch_fill"] == min(8, -(-len(a) // (rounds * S)))
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("slots,integer", [(64, False), (64, True), (8, False)])
def test_measured_batch_layout_rebuilds_equal_oracle(slots, integer):
    """Option balance (default on): from the second build on, batches are cut and ordered by the
    sources' costs measured from the previous builds' batch times -- 300 rows on 64 slots run one
    round (runs of the grouping order sized to equal predicted time), on 8 slots several rounds
    (batches dequeued longest predicted first).  Every rebuild equals the oracle bit for bit."""
    top, g = synthetic_pair(seed=37, n_routers=3000, n_poi=150, n_edges=30000, integer=integer)
    top.set_option("slots", slots)
    top.set_option("tie_dense", 0)  # the batch kernel path (no tie probe)
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    oa, olat, orel, ohops = g.table(verts)
    sizes = set()
    for rep in range(4):
        if rep:
            top.rebuild()
        a, lat, rel, hops = top.table()
        st = top.stats()
        assert st["errors"] == 0
        assert st["batch_layout_measured"] == (1 if rep else 0)
        assert 0 < st["batches"] and (slots == 8 or st["batches"] <= slots)
        sizes.add(st["batches"])
        assert np.array_equal(a, oa)
        assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
        assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
        assert np.array_equal(hops, ohops.astype(np.uint16))
    top.set_option("balance", 0)
    top.rebuild()
    a, lat, rel, hops = top.table()
    assert top.stats()["batch_layout_measured"] == 0
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


def test_sssp_rows_shard_equals_full():
    """build_rows on a row range == the same rows of the full table (sharding correctness)."""
    import torch
    top, g = synthetic_pair(seed=5, n_routers=1500, n_poi=80, n_edges=15000)
    attach_hosts(top, g, 200, type_hints=["client", "relay"])
    a, lat, rel, hops = top.table()
    A = len(a)
    r0, r1 = A // 3, A // 3 + A // 4
    lr = torch.empty((r1 - r0, A, 2), dtype=torch.float64, device="cuda")
    hp = torch.empty((r1 - r0, A), dtype=torch.int16, device="cuda")
    rm = torch.empty((r1 - r0,), dtype=torch.float64, device="cuda")
    top.build_rows_into(r0, r1, lr, hp, rm)
    torch.cuda.synchronize()
    lr = lr.cpu().numpy()
    assert np.array_equal(lr[..., 0].view(np.uint64), lat[r0:r1].view(np.uint64))
    assert np.array_equal(lr[..., 1].view(np.uint64), rel[r0:r1].view(np.uint64))
    assert np.array_equal(hp.cpu().numpy().view(np.uint16), hops[r0:r1])
    assert np.array_equal(rm.cpu().numpy(), lat[r0:r1].min(axis=1))


def test_packet_route_device_vs_oracle():
    """packet_route_kernel vs worker_schedulePacket restatement (seeded drop, delivery time)."""
    import torch
    top, g = bundled_pair("topology")
    geos = list(g.vattrs["geocode"])
    attach_hosts(top, g, g.V, geo_hints=geos)
    a, lat, rel, hops = top.table()
    A = len(a)
    rng = np.random.default_rng(3)
    n = 200_000
    src = rng.integers(0, A, n).astype(np.int32)
    dst = rng.integers(0, A, n).astype(np.int32)
    pay = np.where(rng.random(n) < 0.8, 1448, 0).astype(np.uint32)
    sin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    now = rng.integers(10**9, 2 * 10**9, n).astype(np.uint64)
    jump = 7_000_000
    dev = lambda x: torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else
                                     (x.view(np.int32) if x.dtype == np.uint32 else x)).cuda()
    t_out = torch.empty(n, dtype=torch.int64, device="cuda")
    s_out = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
    top.route_batch_device(dev(src), dev(dst), dev(pay), dev(sin), dev(now), jump, 1, t_out,
                           s_out, d_out)
    torch.cuda.synchronize()
    ot, od, os_ = oracle.route_packets(lat[src, dst], rel[src, dst], pay, sin, now, jump, 1)
    assert np.array_equal(d_out.cpu().numpy(), od)
    assert np.array_equal(t_out.cpu().numpy().view(np.uint64), ot)
    assert np.array_equal(s_out.cpu().numpy().view(np.uint32), os_)
    assert 0 < od.mean() < 1


def test_route_packet_batch_host_api():
    """topology_routePacketBatch (host buffers, IP addressed) vs the oracle."""
    top, g = bundled_pair("topology.plab")
    geos = list(g.vattrs["geocode"])
    otop, ips, verts = attach_hosts(top, g, g.V, geo_hints=geos)
    rng = np.random.default_rng(9)
    n = 5000
    si = rng.integers(0, len(ips), n)
    di = rng.integers(0, len(ips), n)
    src_ip = np.array(ips, dtype=np.uint32)[si]
    dst_ip = np.array(ips, dtype=np.uint32)[di]
    pay = np.where(rng.random(n) < 0.8, 1448, 0).astype(np.uint32)
    sin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    now = rng.integers(10**9, 2 * 10**9, n).astype(np.uint64)
    t, dl, st = top.routePacketBatch(src_ip, dst_ip, pay, sin, now, 3_000_000, True)
    lat = np.array([otop.get_latency(int(a), int(b)) for a, b in zip(src_ip, dst_ip)])
    rel = np.array([otop.get_reliability(int(a), int(b)) for a, b in zip(src_ip, dst_ip)])
    ot, od, os_ = oracle.route_packets(lat, rel, pay, sin, now, 3_000_000, 1)
    assert np.array_equal(dl, od) and np.array_equal(t, ot) and np.array_equal(st, os_)


@pytest.mark.parametrize("integer", [False, True])
def test_lazy_getters_match_reference_cache(integer):
    """topology_getLatency/getReliability with first-rooted-wins emulation vs the reference's
    lazy two-level cache (shd-topology.c:876-938) on one query sequence, incl. the min trajectory."""
    top, g = synthetic_pair(seed=3, n_routers=1200, n_poi=60, n_edges=12000, integer=integer)
    otop, ips, verts = attach_hosts(top, g, 120, type_hints=["client", "relay"])
    shim = sa.topology.shim()
    shim.shim_reset()
    rng = np.random.default_rng(21)
    addrs = {ip: sa.Address(ip) for ip in ips}
    mins = []
    for q in range(600):
        a, b = (int(x) for x in rng.choice(ips, 2))
        l1 = top.getLatency(addrs[a], addrs[b])
        r1 = top.getReliability(addrs[a], addrs[b])
        l2 = otop.get_latency(a, b)
        r2 = otop.get_reliability(a, b)
        assert l1 == l2, (q, l1, l2)
        assert r1 == r2, (q, r1, r2)
        mins.append((top.lazyMinimumLatency(), otop.minimum_path_latency))
    assert all(x == y for x, y in mins)
    assert shim.shim_last_min_latency() == otop.minimum_path_latency


def test_minimum_latency_simple_config1():
    """config 1: the 2-host tgen example (seed chain of SURVEY.md 8(d) C1)."""
    data_top, g = bundled_pair("topology.simple")
    shim = sa.topology.shim()
    master = sa.Random(1)
    slave = sa.Random(master.nextInt())
    hosts = []
    for k in range(2):
        r = sa.Random(slave.nextInt())
        addr = sa.Address("11.0.0.%d" % (k + 1))
        data_top.attach(addr, r)
        hosts.append(addr)
    assert data_top.getLatency(hosts[0], hosts[1]) == 50.0
    assert data_top.getReliability(hosts[0], hosts[1]) == 1.0
    assert data_top.getLatency(hosts[0], hosts[0]) == 20.0
    assert data_top.getMinimumLatency() == 20.0


def _oracle_threads():
    import os
    return max(1, min(64, (os.cpu_count() or 8)))


@pytest.fixture(scope="module")
def c4_table():
    """BASELINE config 4 at full size (1M vertices / 10M edges, the bench workload): the whole
    attached-vertex table built once for the tests below."""
    import torch
    top = sa.Topology.synthetic(seed=20261015)
    assert top.num_vertices == 1_000_000 and top.num_edges == 10_000_000
    top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)  # attaches the C5 hosts
    att = top.attached_vertices()
    A = len(att)
    lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
    hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
    rm = torch.empty((A,), dtype=torch.float64, device="cuda")
    top.build_rows_into(0, A, lr, hp, rm)
    torch.cuda.synchronize()
    rows = np.sort(np.random.default_rng(20261015).choice(A, 128, replace=False))
    yield dict(top=top, att=att, lr=lr, hp=hp, rm=rm, st=top.stats(), rows=rows,
               graph=top.export_graph())
    del lr, hp, rm
    torch.cuda.empty_cache()


def test_sssp_full_size_c4_sampled_rows(c4_table):
    """BASELINE config 4 at full size: 128 seeded rows bit-exact against the oracle's Dijkstra +
    helper (the box's host cores run them in a few seconds), and size-independent properties of
    the whole 10,000 x 10,000 table: every latency finite and > 0, reliability in (0, 1], the
    diagonal is the self loop (1 hop), no overflow fallback, nothing to replay, and the kernel's
    row minima equal the table's."""
    import torch
    att, lr, hp, rm, st, rows = (c4_table[k] for k in ("att", "lr", "hp", "rm", "st", "rows"))
    A = len(att)
    assert st["errors"] == 0 and st["ambiguous_pairs"] == 0 and st["far_scan_sources"] == 0
    assert st["replay_rows"] == 0
    lat = lr[..., 0]
    rel = lr[..., 1]
    assert bool(torch.isfinite(lat).all()) and bool((lat > 0).all())
    assert bool((rel > 0).all()) and bool((rel <= 1).all())
    diag = torch.arange(A, device="cuda")
    assert bool((hp[diag, diag] == 1).all()) and bool((hp >= 1).all())
    assert torch.equal(rm, lat.min(dim=1).values)
    V, eu, ev, elat, eloss, vloss = c4_table["graph"]
    g = oracle.OGraph(V, eu, ev, elat, eloss, vloss)
    olat, orel, ohops = g.source_rows(att[rows], att, nthreads=_oracle_threads())
    glr = lr[torch.from_numpy(rows).cuda()].cpu().numpy()
    assert np.array_equal(glr[..., 0].view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(glr[..., 1].view(np.uint64), orel.view(np.uint64))
    ghp = hp[torch.from_numpy(rows).cuda()].cpu().numpy().view(np.uint16)
    assert np.array_equal(ghp, ohops.astype(np.uint16))


@pytest.mark.timeout(600)
def test_sssp_full_size_c4_rows_vs_scipy(c4_table):
    """BASELINE config 4 at full size, pinned by an implementation independent of the oracle:
    16 of the 128 sampled sources, every one of their 10,000 targets, against scipy's Dijkstra
    predecessor trees + the reference helper (helpers.scipy_rows).  C4's latencies are continuous, so
    every shortest path is unique (the build flags no d-tied parent: ambiguous_pairs == 0) and
    scipy's tree is igraph's; latency, reliability and hops bit for bit.  (Ties stay "parity
    unpinned": DESIGN.md 2.)"""
    import torch
    att, lr, hp, rows, st = (c4_table[k] for k in ("att", "lr", "hp", "rows", "st"))
    assert st["ambiguous_pairs"] == 0
    sub = rows[:: len(rows) // 16][:16]
    slat, srel, shops = scipy_rows(c4_table["graph"], att[sub], att)
    idx = torch.from_numpy(sub).cuda()
    glr = lr[idx].cpu().numpy()
    ghp = hp[idx].cpu().numpy().view(np.uint16)
    assert np.array_equal(glr[..., 0].view(np.uint64), slat.view(np.uint64))
    assert np.array_equal(glr[..., 1].view(np.uint64), srel.view(np.uint64))
    assert np.array_equal(ghp, shops.astype(np.uint16))


def test_sssp_full_size_c4_int_rows():
    """C4-int at full size (1M vertices / 10M edges, integer latencies U{1..100}: 45 % of the
    table's pairs cross a d-tied parent): 64 consecutive rows through the batch kernel + heap
    replay, every pair bit-exact against the oracle (latency, reliability, hops)."""
    import torch
    top = sa.Topology.synthetic(seed=20261015, integer_latency=True)
    top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)
    att = top.attached_vertices()
    A = len(att)
    r0, r1 = 4000, 4064
    lr = torch.empty((r1 - r0, A, 2), dtype=torch.float64, device="cuda")
    hp = torch.empty((r1 - r0, A), dtype=torch.int16, device="cuda")
    top.build_rows_into(r0, r1, lr, hp)
    torch.cuda.synchronize()
    st = top.stats()
    assert st["errors"] == 0 and st["ambiguous_pairs"] > 0 and st["replay_rows"] > 0
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    g = oracle.OGraph(V, eu, ev, elat, eloss, vloss)
    olat, orel, ohops = g.source_rows(att[r0:r1], att, nthreads=_oracle_threads())
    glr = lr.cpu().numpy()
    assert np.array_equal(glr[..., 0].view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(glr[..., 1].view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hp.cpu().numpy().view(np.uint16), ohops.astype(np.uint16))
    # latencies pinned independently of the oracle: with integer edge latencies every shortest
    # path sums to the same exact value whichever tie igraph's heap picks, so scipy's Dijkstra
    # (helpers.scipy_rows) gives the reference's latency bit for bit on 8 of the rows (its
    # reliability and hops follow scipy's own tie choice: not compared)
    sub = np.arange(0, r1 - r0, 8)
    slat, _, _ = scipy_rows((V, eu, ev, elat, eloss, vloss), att[r0 + sub], att)
    assert np.array_equal(glr[sub, :, 0].view(np.uint64), slat.view(np.uint64))


def test_sssp_full_size_c4_dir_rows():
    """C4-dir at full size: the C4 generator with every non-loop edge as two arcs of independent
    latency (1M vertices / 19.99M arcs, igraph mode OUT).  64 rows through the batch kernel --
    out-rows relaxed, parents found in the in-rows -- every pair bit-exact against the oracle's
    directed Dijkstra + helper (latency, reliability, hops); continuous latencies, so nothing is
    replayed."""
    import torch
    top = sa.Topology.synthetic(seed=20261015, directed=True)
    assert top.is_directed and top.num_edges == 2 * 10_000_000 - 10_000
    top.synth_packets(20261015, 100_000, 1000, 10**9, 10**7)
    att = top.attached_vertices()
    A = len(att)
    r0, r1 = 2000, 2064
    lr = torch.empty((r1 - r0, A, 2), dtype=torch.float64, device="cuda")
    hp = torch.empty((r1 - r0, A), dtype=torch.int16, device="cuda")
    top.build_rows_into(r0, r1, lr, hp)
    torch.cuda.synchronize()
    st = top.stats()
    assert st["errors"] == 0 and st["ambiguous_pairs"] == 0 and st["replay_rows"] == 0
    V, eu, ev, elat, eloss, vloss = top.export_graph()
    g = oracle.OGraph(V, eu, ev, elat, eloss, vloss, directed=True)
    olat, orel, ohops = g.source_rows(att[r0:r1], att, nthreads=_oracle_threads())
    glr = lr.cpu().numpy()
    assert not np.array_equal(glr[:, r0:r1, 0], glr[:, r0:r1, 0].T)  # really directed
    assert np.array_equal(glr[..., 0].view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(glr[..., 1].view(np.uint64), orel.view(np.uint64))
    ghp = hp.cpu().numpy().view(np.uint16)
    assert np.array_equal(ghp, ohops.astype(np.uint16))
    # pinned independently of the oracle: continuous latencies, so every shortest path is unique
    # and scipy's directed predecessor tree is igraph's -- 8 of the rows, latency, reliability and
    # hops bit for bit (helpers.scipy_rows, directed)
    sub = np.arange(0, r1 - r0, 8)
    slat, srel, shops = scipy_rows((V, eu, ev, elat, eloss, vloss), att[r0 + sub], att,
                                   directed=True)
    assert np.array_equal(glr[sub, :, 0].view(np.uint64), slat.view(np.uint64))
    assert np.array_equal(glr[sub, :, 1].view(np.uint64), srel.view(np.uint64))
    assert np.array_equal(ghp[sub], shops.astype(np.uint16))


def _grid_graphml(n=30, n_poi=60, seed=5):
    """A 2-D grid of routers (random latencies) whose highest-degree vertex -- the batch kernel's
    landmark h0 -- sits in a corner with long extra edges, so the landmark bound is loose and
    the kappa-prefix cut keeps long rows: the filter must stay exact when h0 is not central."""
    rng = np.random.default_rng(seed)
    keys = ('<key attr.name="packetloss" attr.type="double" for="edge" id="d9" />'
            '<key attr.name="jitter" attr.type="double" for="edge" id="d8" />'
            '<key attr.name="latency" attr.type="double" for="edge" id="d7" />'
            '<key attr.name="type" attr.type="string" for="node" id="d5" />'
            '<key attr.name="bandwidthup" attr.type="int" for="node" id="d4" />'
            '<key attr.name="bandwidthdown" attr.type="int" for="node" id="d3" />'
            '<key attr.name="geocode" attr.type="string" for="node" id="d2" />'
            '<key attr.name="ip" attr.type="string" for="node" id="d1" />'
            '<key attr.name="packetloss" attr.type="double" for="node" id="d0" />')
    out = ['<?xml version="1.0" encoding="utf-8"?><graphml '
           'xmlns="http://graphml.graphdrawing.org/xmlns">', keys,
           '<graph edgedefault="undirected">']

    def node(name, typ, loss, bw):
        out.append('<node id="%s"><data key="d0">%r</data><data key="d1">0.0.0.0</data>'
                   '<data key="d2">US</data><data key="d3">%d</data><data key="d4">%d</data>'
                   '<data key="d5">%s</data></node>' % (name, loss, bw, bw, typ))

    def edge(a, b, lat, loss):
        out.append('<edge source="%s" target="%s"><data key="d7">%r</data>'
                   '<data key="d8">0</data><data key="d9">%r</data></edge>' % (a, b, lat, loss))

    for i in range(n * n):
        node("pop-%d" % i, "pop", 0.0, 0)
    for k in range(n_poi):
        node("poi-%d" % k, ("client", "relay", "server")[k % 3],
             float(rng.uniform(0, 0.05)), 10240)
    for r in range(n):
        for c in range(n):
            i = r * n + c
            if c + 1 < n:
                edge("pop-%d" % i, "pop-%d" % (i + 1), float(rng.uniform(1, 100)),
                     float(rng.uniform(0, 0.01)))
            if r + 1 < n:
                edge("pop-%d" % i, "pop-%d" % (i + n), float(rng.uniform(1, 100)),
                     float(rng.uniform(0, 0.01)))
    for t in rng.choice(np.arange(1, n * n), 24, replace=False):  # corner hub, long edges
        edge("pop-0", "pop-%d" % t, float(rng.uniform(150, 400)), 0.0)
    for k in range(n_poi):
        edge("poi-%d" % k, "pop-%d" % int(rng.integers(0, n * n)), 5.0, 0.0)
        edge("poi-%d" % k, "poi-%d" % k, 1.0, 0.0)
    out.append("</graph></graphml>")
    return "".join(out).encode()


@pytest.mark.parametrize("hubs", [-1, 0])
def test_sssp_batch_peripheral_landmark(hubs):
    """Landmark filter / kappa cut / tree-parent guesses on a grid whose landmark is peripheral:
    every pair bit-exact against the oracle."""
    data = _grid_graphml()
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    assert not top.is_complete
    top.set_option("lds_hubs", hubs)
    top.set_option("batch", 8)
    top.set_option("batch_fill", 8)
    otop, ips, verts = attach_hosts(top, g, 60, type_hints=["client", "relay", "server"])
    a, lat, rel, hops = top.table()
    st = top.stats()
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert st["errors"] == 0 and st["ambiguous_pairs"] == 0
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))


def test_lds_hubs_lowered_between_builds():
    """a launch copies its hub distances into rows [0, H) of every slot's [V][K] block
    (the epilogue).  A later launch with fewer LDS hubs treats vertices [H', H) as tail vertices,
    whose lines must start at +inf: the library refills them before such a launch.  Build with
    every hub in LDS, lower lds_hubs (two steps), rebuild: every table equals the oracle's."""
    top, g = synthetic_pair(seed=13, n_routers=3000, n_poi=150, n_edges=30000)
    top.set_option("batch_fill", 8)
    top.set_option("slots", 4)  # few slots: every slot's block serves several batches
    otop, ips, verts = attach_hosts(top, g, 300, type_hints=["client", "relay", "server"])
    oa, olat, orel, ohops = g.table(verts)
    seen = []
    for hubs in (-1, 600, 0):
        top.set_option("lds_hubs", hubs)
        top.rebuild()
        a, lat, rel, hops = top.table()
        st = top.stats()
        seen.append(st["lds_hubs"])
        assert st["errors"] == 0
        assert np.array_equal(a, oa)
        assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
        assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
        assert np.array_equal(hops, ohops.astype(np.uint16))
    assert seen[0] > seen[1] > seen[2] == 0


def test_device_option_after_topology_new_builds_on_that_device(tmp_path):
    """topology_new initialises the default device in the background while it parses (the HIP
    context, queues and code objects: ~150 ms off the first build).  Setting "device" before the
    first attach releases that init and the next use initialises the chosen device (on the
    one-GPU test box every ordinal maps to device 0, so the move is observed by the second
    initialisation); the table built there equals the oracle's."""
    import time
    import torch
    syn = sa.Topology.synthetic(seed=19, n_routers=2000, n_poi=100, n_edges=20000)
    path = str(tmp_path / "t.graphml.xml")
    syn.write_graphml(path)
    syn.free()
    top = sa.Topology.new(path)
    g = oracle.OGraph.from_graphml(path)
    t0 = time.time()
    while top.stats()["dev_inits"] < 1 and time.time() - t0 < 60:
        time.sleep(0.05)
    assert top.stats()["dev_inits"] == 1 and top.stats()["init_bg_ms"] > 0
    top.set_option("device", torch.cuda.device_count())  # another ordinal (maps to 0 here)
    otop, ips, verts = attach_hosts(top, g, 200, type_hints=["client", "relay"])
    with pytest.raises(KeyError):
        top.set_option("device", 0 if torch.cuda.device_count() > 1 else 1 + torch.cuda.device_count())
    a, lat, rel, hops = top.table()
    assert top.stats()["dev_inits"] == 2
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(a, oa)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("integer", [False, True])
def test_repeated_one_round_builds_equal_oracle(integer):
    """A one-round launch (fewer batches than workgroups) rebuilt four times -- the measured batch
    layout (option balance) takes over from the second build, so the batches change -- stays bit
    for bit the first build and the oracle's table, with no failed pair.  (Round 5 ran the same
    builds with the help board, which round 6 removed: DESIGN.md 4 item 10.)"""
    top, g = synthetic_pair(seed=43, n_routers=20000, n_poi=400, n_edges=200000, integer=integer)
    top.set_option("tie_dense", 0)
    otop, ips, verts = attach_hosts(top, g, 1200, type_hints=["client", "relay", "server"])
    a0, lat0, rel0, hops0 = top.table()
    for rep in range(4):
        top.rebuild()
        a, lat, rel, hops = top.table()
        st = top.stats()
        assert st["errors"] == 0
        assert np.array_equal(a, a0)
        assert np.array_equal(lat.view(np.uint64), lat0.view(np.uint64))
        assert np.array_equal(rel.view(np.uint64), rel0.view(np.uint64))
        assert np.array_equal(hops, hops0)
    assert top.stats()["batch_layout_measured"] == 1
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat0.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel0.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops0, ohops.astype(np.uint16))


@pytest.mark.parametrize("integer", [False, True])
def test_row_scans_in_small_chunks_equal_oracle(integer):
    """The parent pass scans the rows of the pairs whose recorded parents failed (R) in chunks of
    row_scan_chunk pairs, with one scan record per (merged vertex, source) of a chunk (round 6:
    the [V][K] best / cnt / bslot arrays, 32 GB at C4, became 16 B x K per pair of a chunk).
    With no hub parent hints (par_hubs 0: every hub pair is scanned) and 64-pair chunks, a level
    takes many chunks and a vertex's sources fall into several; the tables equal the default
    chunk's and the oracle's, bit for bit."""
    top, g = synthetic_pair(seed=53, n_routers=20000, n_poi=300, n_edges=200000, integer=integer)
    top.set_option("tie_dense", 0)
    top.set_option("par_hubs", 0)
    otop, ips, verts = attach_hosts(top, g, 900, type_hints=["client", "relay", "server"])
    a0, lat0, rel0, hops0 = top.table()
    st = top.stats()
    assert st["errors"] == 0
    n_batches = (len(verts) + 7) // 8
    # pairs sent to row scans: several 64-pair chunks per batch
    assert st["walk_kinds"][3] > 2 * 64 * n_batches, st["walk_kinds"]
    with pytest.raises(KeyError):
        top.set_option("row_scan_chunk", 63)
    top.set_option("row_scan_chunk", 64)
    top.rebuild()
    a, lat, rel, hops = top.table()
    assert top.stats()["errors"] == 0
    assert np.array_equal(a, a0)
    assert np.array_equal(lat.view(np.uint64), lat0.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), rel0.view(np.uint64))
    assert np.array_equal(hops, hops0)
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops, ohops.astype(np.uint16))


@pytest.mark.parametrize("n_hosts", [1, 2, 9, 17])
def test_small_and_ragged_attached_sets_equal_oracle(n_hosts):
    """Edge sizes of the batch launch: one attached host (a 1 x 1 table: the self pair through
    the self loop), two, and counts that leave a ragged last batch (9 = 8 + 1, 17 = 2 x 8 + 1),
    under the default options (auto batch fill, measured layout from the second build on) --
    first build and a rebuild, both bit for bit the oracle's."""
    top, g = synthetic_pair(seed=59, n_routers=3000, n_poi=150, n_edges=30000)
    top.set_option("tie_dense", 0)
    otop, ips, verts = attach_hosts(top, g, n_hosts, type_hints=["client", "relay", "server"])
    oa, olat, orel, ohops = g.table(verts)
    for rep in range(2):
        if rep:
            top.rebuild()
        a, lat, rel, hops = top.table()
        assert top.stats()["errors"] == 0
        assert np.array_equal(a, oa)
        assert np.array_equal(lat.view(np.uint64), olat.view(np.uint64))
        assert np.array_equal(rel.view(np.uint64), orel.view(np.uint64))
        assert np.array_equal(hops, ohops.astype(np.uint16))
    assert top.getMinimumLatency() == olat.min()


@pytest.mark.parametrize("integer", [False, True])
def test_bucket_width_and_landmark_phase_do_not_change_the_table(integer):
    """Option delta (bucket width) and h0_phase (where the landmark h0 sits in its bucket; < 0 the
    round-4 shifts) change only the order of the label-correcting work, not the fixpoint: tables
    built with several settings on one topology are bit-identical, and equal the oracle's."""
    top, g = synthetic_pair(seed=47, n_routers=20000, n_poi=300, n_edges=200000, integer=integer)
    top.set_option("tie_dense", 0)
    otop, ips, verts = attach_hosts(top, g, 900, type_hints=["client", "relay", "server"])
    a0, lat0, rel0, hops0 = top.table()
    assert top.stats()["errors"] == 0
    for delta, phase in ((10.1, -1.0), (25.0, 0.3), (80.0, 0.98), (5.0, 0.5)):
        top.set_option("delta", delta)
        top.set_option("h0_phase", phase)
        top.rebuild()
        a, lat, rel, hops = top.table()
        assert top.stats()["errors"] == 0
        assert np.array_equal(a, a0)
        assert np.array_equal(lat.view(np.uint64), lat0.view(np.uint64)), (delta, phase)
        assert np.array_equal(rel.view(np.uint64), rel0.view(np.uint64)), (delta, phase)
        assert np.array_equal(hops, hops0), (delta, phase)
    oa, olat, orel, ohops = g.table(verts)
    assert np.array_equal(lat0.view(np.uint64), olat.view(np.uint64))
    assert np.array_equal(rel0.view(np.uint64), orel.view(np.uint64))
    assert np.array_equal(hops0, ohops.astype(np.uint16))
