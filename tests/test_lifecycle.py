"""GPU parity of the engine-faithful adapter over a topology's life: late attaches, detaches,
the lazy per-window packet batch and the reference's own tcp fixtures, each against the
reference Topology restatement (oracle.OracleTopology: the two-level path cache of
shd-topology.c:434-512,876-963, whose target set is the attached set at the moment a row is
computed, :690-744).
"""
import json
import os

import numpy as np
import pytest

import oracle
import shadow_amd as sa
from helpers import host_ip, synthetic_pair

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def attach_range(top, otop, k0, n, seed, hints=("client", "relay", "server")):
    """Attach hosts k0..k0+n-1 to both topologies with identical rand_r streams."""
    ips = []
    st = seed
    for k in range(k0, k0 + n):
        st = (st * 1103515245 + 12345) & 0xFFFFFFFF
        ip = host_ip(k + 1)
        v1, s1 = top.attach_ip(ip, st, typeHint=hints[k % len(hints)])
        v2, s2 = otop.attach(ip, st, type_hint=hints[k % len(hints)])
        assert v1 == v2 and s1 == s2
        ips.append(ip)
    return ips


def query_both(top, otop, rng, ips, n, shim):
    for q in range(n):
        a, b = (int(x) for x in rng.choice(ips, 2))
        r1 = top.reliability_ip(a, b)
        l1 = top.latency_ip(a, b)
        r2 = otop.get_reliability(a, b)
        l2 = otop.get_latency(a, b)
        assert l1 == l2 and r1 == r2, (q, a, b, l1, l2, r1, r2)
        assert top.lazyMinimumLatency() == otop.minimum_path_latency, q
    # the engine sees the same minimum (the number of pushes inside one computed row follows
    # GLib's hash order of the target set, shd-topology.c:690-744: not part of the contract)
    assert shim.shim_last_min_latency() == otop.minimum_path_latency


@pytest.mark.parametrize("integer", [True, False])
def test_late_attach_and_detach_match_reference_cache(integer):
    """Queries, then late attaches (onto new vertices: the reference recomputes rows on a miss
    and may push a lower minimum), then detaches (cached paths stay, the target set shrinks for
    rows computed afterwards), then a re-attach: every answer and the min trajectory (values
    after every query, and the value the engine last received) equal the reference cache's."""
    top, g = synthetic_pair(seed=4, n_routers=1500, n_poi=90, n_edges=15000, integer=integer)
    shim = sa.topology.shim()
    shim.shim_reset()
    otop = oracle.OracleTopology(g)
    rng = np.random.default_rng(5)
    ips = attach_range(top, otop, 0, 40, seed=7)
    query_both(top, otop, rng, ips, 150, shim)
    # late attaches: many land on vertices no earlier host used
    new = attach_range(top, otop, 40, 40, seed=99)
    assert len(set(otop.virtual_ip.values())) > len(set(otop.virtual_ip[i] for i in ips))
    ips += new
    query_both(top, otop, rng, ips, 300, shim)
    # detaches: half of the early hosts; some were alone on their vertex
    gone = ips[:40:2]
    for ip in gone:
        top.detach_ip(ip)
        otop.detach(ip)
    live = [ip for ip in ips if ip not in set(gone)]
    for ip in gone[:3]:
        assert top.latency_ip(ip, live[0]) == -1.0 and otop.get_latency(ip, live[0]) == -1.0
    query_both(top, otop, rng, live, 300, shim)
    assert len(top.attached_vertices()) == len(set(otop.virtual_ip.values()))
    # a detached address attaches again (maybe elsewhere)
    again = attach_range(top, otop, 0, 1, seed=12345)
    live += again
    query_both(top, otop, rng, live, 200, shim)


def test_build_rows_after_detach_uses_current_geometry():
    """shdtopo_build_rows after a detach: the table and the getters follow the new columns (no
    stale A x A table indexed with the new column map)."""
    import torch
    top, g = synthetic_pair(seed=6, n_routers=1200, n_poi=60, n_edges=12000)
    otop = oracle.OracleTopology(g)
    ips = attach_range(top, otop, 0, 50, seed=3)
    a0, lat0, _, _ = top.table()
    # detach every host of one vertex
    v0 = otop.virtual_ip[ips[0]]
    for ip in [i for i in ips if otop.virtual_ip.get(i) == v0]:
        top.detach_ip(ip)
        otop.detach(ip)
    att = top.attached_vertices()
    assert len(att) == len(a0) - 1 and v0 not in set(att.tolist())
    A = len(att)
    lr = torch.empty((A, A, 2), dtype=torch.float64, device="cuda")
    hp = torch.empty((A, A), dtype=torch.int16, device="cuda")
    top.build_rows_into(0, A, lr, hp)
    torch.cuda.synchronize()
    keep = np.isin(a0, att)
    assert np.array_equal(lr[..., 0].cpu().numpy(), lat0[np.ix_(keep, keep)])
    live = [ip for ip in ips if ip in otop.virtual_ip]
    for x, y in zip(live[:40], live[1:41]):
        assert top.latency_ip(x, y) == otop.get_latency(x, y)


@pytest.mark.parametrize("integer", [True, False])
def test_route_packet_batch_lazy_sssp_vs_reference(integer):
    """topology_routePacketBatch in lazy mode on an SSSP graph where orientation matters: every
    packet (delivered, time, state) equals worker_schedulePacket over the reference cache in
    emission order (getReliability, draw, getLatency: shd-worker.c:352-361), and so does the
    running minimum."""
    top, g = synthetic_pair(seed=8, n_routers=1500, n_poi=80, n_edges=15000, integer=integer)
    shim = sa.topology.shim()
    shim.shim_reset()
    otop = oracle.OracleTopology(g)
    ips = attach_range(top, otop, 0, 120, seed=11)
    rng = np.random.default_rng(13)
    n = 4000
    si = np.asarray(ips, np.uint32)[rng.integers(0, len(ips), n)]
    di = np.asarray(ips, np.uint32)[rng.integers(0, len(ips), n)]
    pay = np.where(rng.random(n) < 0.8, 1448, 0).astype(np.uint32)
    sin = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    now = rng.integers(10**9, 2 * 10**9, n).astype(np.uint64)
    jump = 4_000_000
    t, dl, st = top.routePacketBatch(si, di, pay, sin, now, jump, True)
    rel = np.array([otop.get_reliability(int(a), int(b)) for a, b in zip(si, di)])
    lat = np.array([otop.get_latency(int(a), int(b)) for a, b in zip(si, di)])
    ot, od, os_ = oracle.route_packets(lat, rel, pay, sin, now, jump, 1)
    assert np.array_equal(dl, od) and np.array_equal(t, ot) and np.array_equal(st, os_)
    assert top.lazyMinimumLatency() == otop.minimum_path_latency
    assert shim.shim_last_min_latency() == otop.minimum_path_latency
    assert top.stats()["route_bad_packets"] == 0


@pytest.mark.parametrize("name", ["lossless", "lossy"])
def test_tcp_fixture_topologies_through_hip(name, tmp_path):
    """The reference's own topology fixtures (src/test/tcp/*.test.shadow.config.xml:14-26, one
    vertex, 50 ms self loop, loss 0 / 0.25) through topology_new (file path) + topology_attach
    + the getters on the GPU path: (50.0, 1.0) / (50.0, 0.75)."""
    d = json.load(open(os.path.join(GOLDEN, "tcp_1vertex.json")))[name]
    path = tmp_path / "tcp.graphml.xml"
    path.write_text(d["graphml"])
    top = sa.Topology.new(str(path))
    assert top is not None and top.is_complete and top.num_vertices == 1
    master = sa.Random(1)
    slave = sa.Random(master.nextInt())
    client, server = sa.Address("11.0.0.1"), sa.Address("11.0.0.2")
    for a in (client, server):
        top.attach(a, sa.Random(slave.nextInt()))
    assert top.getLatency(client, server) == 50.0 == d["latency"]
    assert top.getReliability(client, server) == d["reliability"]
    assert top.getReliability(client, server) == (0.75 if name == "lossy" else 1.0)
    assert top.isRoutable(client, server)
    assert top.getMinimumLatency() == 50.0
    stranger = sa.Address("11.0.0.9")
    assert top.getLatency(client, stranger) == -1.0 and not top.isRoutable(stranger, client)


def test_packet_route_full_c5_window():
    """BASELINE config 5 at full size: the bench's 10,000,000-packet Tor-like window (100,000
    hosts on C4's 9,999 attached poi) routed on the GPU over the full C4 table; every packet's
    delivered flag, delivery time and new rand_r state equal the oracle's."""
    import torch
    top = sa.Topology.synthetic(seed=20261015)
    pk = top.synth_packets(20261015, 100_000, 10_000_000, 10**9, 10**7)
    a, lat, rel, hops = top.table()
    gmin = top.getMinimumLatency()
    jump = int(gmin) * 1_000_000
    cu = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    n = len(pk["src_col"])
    t_out = torch.empty(n, dtype=torch.int64, device="cuda")
    s_out = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
    top.route_batch_device(cu(pk["src_col"]), cu(pk["dst_col"]), cu(pk["payload"].view(np.int32)),
                           cu(pk["state_in"].view(np.int32)), cu(pk["now"].view(np.int64)), jump,
                           1, t_out, s_out, d_out)
    torch.cuda.synchronize()
    s, d = pk["src_col"], pk["dst_col"]
    ot, od, os_ = oracle.route_packets(lat[s, d], rel[s, d], pk["payload"], pk["state_in"],
                                       pk["now"], jump, 1)
    assert np.array_equal(d_out.cpu().numpy(), od)
    assert np.array_equal(t_out.cpu().numpy().view(np.uint64), ot)
    assert np.array_equal(s_out.cpu().numpy().view(np.uint32), os_)
    assert 0.5 < od.mean() < 1.0 and top.stats()["route_bad_packets"] == 0


def test_packet_route_rejects_bad_columns():
    """Columns outside [0, A) are not routed (no out-of-bounds gather) and are counted."""
    import torch
    top, g = synthetic_pair(seed=2, n_routers=800, n_poi=40, n_edges=8000)
    otop = oracle.OracleTopology(g)
    attach_range(top, otop, 0, 60, seed=1)
    a, lat, rel, hops = top.table()
    A = len(a)
    src = torch.tensor([0, A, -1, 1, A + 5], dtype=torch.int32, device="cuda")
    dst = torch.tensor([1, 0, 0, 10**6, 2], dtype=torch.int32, device="cuda")
    n = 5
    z32 = torch.zeros(n, dtype=torch.int32, device="cuda")
    st_in = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    now = torch.full((n,), 10**9, dtype=torch.int64, device="cuda")
    t_out = torch.empty(n, dtype=torch.int64, device="cuda")
    s_out = torch.empty(n, dtype=torch.int32, device="cuda")
    d_out = torch.empty(n, dtype=torch.uint8, device="cuda")
    top.route_batch_device(src, dst, z32, st_in, now, 0, 0, t_out, s_out, d_out)
    torch.cuda.synchronize()
    assert d_out.cpu().tolist() == [1, 0, 0, 0, 0]
    assert s_out.cpu().tolist()[1:] == [7, 7, 7, 7]
    assert top.stats()["route_bad_packets"] == 4
