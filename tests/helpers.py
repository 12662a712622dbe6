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
