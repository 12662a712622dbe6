"""The product window adapter (include/shd_topology_window.h) against the reference's per-packet
worker_schedulePacket (src/engine/shd-worker.c:332-370) over the reference Topology restatement
(oracle.OracleTopology), in multi-threaded windows (runahead clamp) and serial-mode windows.

Hosts carry Shadow Random streams (libshdtopo_shim.so); packets go through topowindow_emit, which
captures the pre-draw state and takes the draw, and come back through topowindow_flush's deliver
callback.  The reference side replays the same emission order with getReliability, the draw,
getLatency and the clamp.
"""
import math

import numpy as np
import pytest

import oracle
import shadow_amd as sa
from shadow_amd import _lib
from helpers import host_ip, synthetic_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("serial", [False, True])
def test_window_adapter_vs_reference(serial):
    top, g = synthetic_pair(seed=31, n_routers=1500, n_poi=80, n_edges=15000, integer=True)
    lib, shim = _lib.load()
    otop = oracle.OracleTopology(g)
    nh = 150
    hosts = []
    st = 5
    for k in range(nh):
        st = (st * 1103515245 + 12345) & 0xFFFFFFFF
        ip = host_ip(k + 1)
        v1, s1 = top.attach_ip(ip, st, typeHint=("client", "relay", "server")[k % 3])
        v2, s2 = otop.attach(ip, st, type_hint=("client", "relay", "server")[k % 3])
        assert v1 == v2 and s1 == s2
        hosts.append((ip, sa.Address(ip), sa.Random(s1)))
    ref_state = [h[2].state for h in hosts]
    w = lib.topowindow_new(top._h)
    jump = lib.topowindow_serial_window_ns(top._h) if serial else lib.topowindow_jump_ns(top._h, 0)
    gmin = top.getMinimumLatency()
    if serial:
        assert jump == math.floor(gmin * 1e6)
    else:
        assert jump == int(gmin) * 1_000_000
    got = {}

    @_lib.WINDOW_DELIVER
    def deliver(ctx, packet, delivered, time):
        got[int(packet)] = (delivered, time)

    rng = np.random.default_rng(8)
    t0 = 10**9
    for win in range(3):
        ref = []
        for k in range(1500):
            s, d = (int(x) for x in rng.choice(nh, 2, replace=False))
            pay = 1448 if rng.random() < 0.8 else 0
            now = t0 + int(rng.integers(0, jump))
            # reference, shd-worker.c:345-369 at emit
            rel = otop.get_reliability(hosts[s][0], hosts[d][0])
            r, ref_state[s] = oracle.next_double(ref_state[s])
            dl = r <= rel or pay == 0
            t = 0
            if dl:
                lat = otop.get_latency(hosts[s][0], hosts[d][0])
                t = now + int(math.ceil(lat * 1e6))
                if not serial:
                    t = max(t, now + jump)
                else:
                    assert t >= t0 + jump  # the deferral changes no arrival time
            ref.append((int(dl), t))
            # adapter
            idx = lib.topowindow_emit(w, hosts[s][1]._p, hosts[d][1]._p, pay, hosts[s][2]._p, now,
                                      k + 1)
            assert idx == k
            assert hosts[s][2].state == ref_state[s]
        got.clear()
        assert lib.topowindow_pending(w) == len(ref)
        assert lib.topowindow_flush(w, jump, 0 if serial else 1, deliver, None) == 0
        assert lib.topowindow_pending(w) == 0
        assert [got[k + 1] for k in range(len(ref))] == ref
        assert top.lazyMinimumLatency() == otop.minimum_path_latency
        t0 += jump
    lib.topowindow_free(w)


def test_window_routes_packets_of_a_host_detached_before_the_flush():
    """a packet is routed at emit in the reference (shd-worker.c:345-369).  A host
    that detaches (the last host on its vertex) after emitting or being sent packets in a window
    keeps its vertex's table column until the window's flush (shdtopo_window_hold / _release),
    so those packets come back exactly as the reference routed them; the column goes after the
    flush (a later query rebuilds the table without it)."""
    top, g = synthetic_pair(seed=33, n_routers=1500, n_poi=80, n_edges=15000)
    lib, shim = _lib.load()
    otop = oracle.OracleTopology(g)
    hosts, verts = [], []
    st = 9
    for k in range(60):
        st = (st * 1103515245 + 12345) & 0xFFFFFFFF
        ip = host_ip(k + 1)
        v1, s1 = top.attach_ip(ip, st, typeHint=("client", "relay")[k % 2])
        v2, s2 = otop.attach(ip, st, type_hint=("client", "relay")[k % 2])
        assert v1 == v2 and s1 == s2
        hosts.append((ip, sa.Address(ip), sa.Random(s1)))
        verts.append(v1)
    # a host alone on its vertex
    lone = next(i for i, v in enumerate(verts) if verts.count(v) == 1)
    A0 = len(top.attached_vertices())
    w = lib.topowindow_new(top._h)
    jump = lib.topowindow_jump_ns(top._h, 0)
    got = {}

    @_lib.WINDOW_DELIVER
    def deliver(ctx, packet, delivered, time):
        got[int(packet)] = (delivered, time)

    ref_state = [h[2].state for h in hosts]
    ref = []
    rng = np.random.default_rng(3)
    t0 = 10**9
    for k in range(400):
        a = lone if k % 2 == 0 else int(rng.integers(0, len(hosts)))
        b = int(rng.integers(0, len(hosts)))
        s, d = (a, b) if k % 4 < 2 else (b, a)
        if s == d:
            d = (d + 1) % len(hosts)
        pay = 1448
        now = t0 + int(rng.integers(0, jump))
        rel = otop.get_reliability(hosts[s][0], hosts[d][0])
        r, ref_state[s] = oracle.next_double(ref_state[s])
        dl = r <= rel
        t = max(now + int(math.ceil(otop.get_latency(hosts[s][0], hosts[d][0]) * 1e6)),
                now + jump) if dl else 0
        ref.append((int(dl), t))
        assert lib.topowindow_emit(w, hosts[s][1]._p, hosts[d][1]._p, pay, hosts[s][2]._p, now,
                                   k + 1) == k
    top.detach_ip(hosts[lone][0])  # the lone host leaves before the window's flush
    assert lib.topowindow_flush(w, jump, 1, deliver, None) == 0
    assert [got[k + 1] for k in range(len(ref))] == ref
    assert any(x[0] for x in ref)
    # after the flush the vertex is no longer a column
    assert len(top.attached_vertices()) == A0 - 1
    lib.topowindow_free(w)


def _near_pair_graphml():
    """A ring of 16 routers (10 ms links) and 12 poi with distinct geocodes: poi 2j and 2j + 1
    share router j (1 ms uplinks, so they are 2 ms apart) and have 100-ms self loops, so a poi's
    nearest attached vertex is its twin, not itself."""
    keys = ('<key attr.name="packetloss" attr.type="double" for="edge" id="d9" />'
            '<key attr.name="latency" attr.type="double" for="edge" id="d7" />'
            '<key attr.name="type" attr.type="string" for="node" id="d5" />'
            '<key attr.name="geocode" attr.type="string" for="node" id="d2" />'
            '<key attr.name="ip" attr.type="string" for="node" id="d1" />'
            '<key attr.name="packetloss" attr.type="double" for="node" id="d0" />')
    out = ['<?xml version="1.0" encoding="utf-8"?><graphml '
           'xmlns="http://graphml.graphdrawing.org/xmlns">', keys,
           '<graph edgedefault="undirected">']
    for i in range(16):
        out.append('<node id="r%d"><data key="d0">0.0</data><data key="d1">0.0.0.0</data>'
                   '<data key="d2">XX</data><data key="d5">pop</data></node>' % i)
    for k in range(12):
        out.append('<node id="poi-%d"><data key="d0">0.001</data><data key="d1">0.0.0.0</data>'
                   '<data key="d2">G%d</data><data key="d5">client</data></node>' % (k, k))
    for i in range(16):
        out.append('<edge source="r%d" target="r%d"><data key="d7">10.0</data>'
                   '<data key="d9">0.0</data></edge>' % (i, (i + 1) % 16))
    for k in range(12):
        out.append('<edge source="poi-%d" target="r%d"><data key="d7">%r</data>'
                   '<data key="d9">0.001</data></edge>' % (k, k // 2, 1.0 + 0.01 * k))
        out.append('<edge source="poi-%d" target="poi-%d"><data key="d7">100.0</data>'
                   '<data key="d9">0.0</data></edge>' % (k, k))
    out.append("</graph></graphml>")
    return "".join(out).encode()


def test_window_lazy_minimum_excludes_a_column_detached_in_the_window():
    """a vertex that loses its last host inside a window keeps its table column until
    the flush, but a source row first computed after the detach must take its minimum over the
    vertices attached at that moment (shd-topology.c:690-744), as the reference's row does.  Here
    the detached poi is the twin (2.01 ms away) of the later source, whose other entries are >= 20
    ms, and the only other computed row's minimum is 2.13 ms (X's twin): the running minimum must
    stay the reference's 2.13, not drop to 2.01."""
    data = _near_pair_graphml()
    top = sa.Topology.from_buffer(data)
    g = oracle.OGraph.from_graphml(data)
    lib, shim = _lib.load()
    otop = oracle.OracleTopology(g)
    hosts = []
    st = 3
    for k in range(12):  # one host per poi (geocode hint)
        st = (st * 1103515245 + 12345) & 0xFFFFFFFF
        ip = host_ip(k + 1)
        v1, s1 = top.attach_ip(ip, st, geocodeHint="G%d" % k)
        v2, s2 = otop.attach(ip, st, geocode_hint="G%d" % k)
        assert v1 == v2 and s1 == s2
        hosts.append((ip, sa.Address(ip), sa.Random(s1)))
    L, S, X, D = 0, 1, 6, 8  # L and S are twins; X, D elsewhere on the ring
    w = lib.topowindow_new(top._h)
    jump = lib.topowindow_jump_ns(top._h, 0)
    got = {}

    @_lib.WINDOW_DELIVER
    def deliver(ctx, packet, delivered, time):
        got[int(packet)] = (delivered, time)

    ref_state = [h[2].state for h in hosts]
    ref = []
    t0 = 10**9

    def emit(k, s, d):
        now = t0 + 1000 * k
        rel = otop.get_reliability(hosts[s][0], hosts[d][0])
        r, ref_state[s] = oracle.next_double(ref_state[s])
        dl = r <= rel
        t = max(now + int(math.ceil(otop.get_latency(hosts[s][0], hosts[d][0]) * 1e6)),
                now + jump) if dl else 0
        ref.append((int(dl), t))
        assert lib.topowindow_emit(w, hosts[s][1]._p, hosts[d][1]._p, 1448, hosts[s][2]._p, now,
                                   k + 1) == k

    emit(0, X, L)  # row X (all 12 columns, L's included) enters the cache
    emit(1, L, X)  # answered from row X: row L is never computed
    top.detach_ip(hosts[L][0])
    otop.detach(hosts[L][0])
    emit(2, S, D)  # row S computed now, over the 11 vertices still attached
    assert lib.topowindow_flush(w, jump, 1, deliver, None) == 0
    assert [got[k + 1] for k in range(len(ref))] == ref
    # the reference's running minimum: row X's and row S's (without L's twin column)
    assert otop.minimum_path_latency > 2.1
    assert top.lazyMinimumLatency() == otop.minimum_path_latency
    lib.topowindow_free(w)
