"""Generate the committed golden fixtures under tests/golden/ from the CPU oracle.

Run from the repo root:  python tests/golden/make_golden.py
(The reference itself cannot be built or imported here -- it needs igraph, SURVEY.md K4 -- so
every fixture is produced by the oracle's restatement and pinned where the reference offers an
anchor: the tcp test topologies' formula values, glibc rand_r, scipy distances.)

Fixtures:
  tcp_1vertex.json      1-vertex topologies of src/test/tcp/*.test.shadow.config.xml (data)
                        with the hand-derived expected (latency, reliability)
  c1_simple.json        config 1: topology.simple + 2 hosts via the seed chain
  bundled_tables.json   configs 2/3: A x A table digests + 1000 sampled entries
  synth_real.npz        1,500-vertex non-complete graph, continuous latencies: 16 SSSP rows
  synth_int.npz         same shape, integer latencies (heavy parent ties)
  packets.npz           1,000 packet-route vectors (shd-worker.c:332-370)
"""
import hashlib
import json
import lzma
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402

TCP_GRAPHML = """<graphml xmlns="http://graphml.graphdrawing.org/xmlns">
  <key attr.name="packetloss" attr.type="double" for="edge" id="d9" />
  <key attr.name="jitter" attr.type="double" for="edge" id="d8" />
  <key attr.name="latency" attr.type="double" for="edge" id="d7" />
  <key attr.name="asn" attr.type="int" for="node" id="d6" />
  <key attr.name="type" attr.type="string" for="node" id="d5" />
  <key attr.name="bandwidthup" attr.type="int" for="node" id="d4" />
  <key attr.name="bandwidthdown" attr.type="int" for="node" id="d3" />
  <key attr.name="geocode" attr.type="string" for="node" id="d2" />
  <key attr.name="ip" attr.type="string" for="node" id="d1" />
  <key attr.name="packetloss" attr.type="double" for="node" id="d0" />
  <graph edgedefault="undirected">
    <node id="poi-1">
      <data key="d0">0.0</data>
      <data key="d1">0.0.0.0</data>
      <data key="d2">US</data>
      <data key="d3">10240</data>
      <data key="d4">10240</data>
      <data key="d5">testnet</data>
      <data key="d6">0</data>
    </node>
    <edge source="poi-1" target="poi-1">
      <data key="d7">50.0</data>
      <data key="d8">0.0</data>
      <data key="d9">%s</data>
    </edge>
  </graph>
</graphml>
"""


def bundled(name):
    with lzma.open(os.path.join(HERE, "resource", name + ".graphml.xml.xz")) as f:
        return f.read()


def synth_graph(seed, R, P, n_cl, integer):
    """Small power-law graph of the C4 shape: Chung-Lu routers + spanning path + poi uplinks and
    self loops (K7).  numpy only, independent of the product's generator."""
    rng = np.random.default_rng(seed)
    w = (rng.permutation(R) + 1.0) ** (-1 / 1.1)
    p = w / w.sum()
    pairs = set()
    perm = rng.permutation(R)
    eu, ev = [], []
    for i in range(R - 1):
        a, b = int(perm[i]), int(perm[i + 1])
        pairs.add((min(a, b), max(a, b)))
        eu.append(a)
        ev.append(b)
    while len(eu) < (R - 1) + n_cl:
        a, b = (int(x) for x in rng.choice(R, 2, p=p))
        if a == b or (min(a, b), max(a, b)) in pairs:
            continue
        pairs.add((min(a, b), max(a, b)))
        eu.append(a)
        ev.append(b)
    m = len(eu)
    lat = rng.integers(1, 101, m).astype(float) if integer else rng.uniform(1, 100, m)
    loss = rng.uniform(0, 0.01, m)
    up = rng.integers(0, R, P)
    eu += list(range(R, R + P)) + list(range(R, R + P))
    ev += [int(x) for x in up] + list(range(R, R + P))
    lat = np.concatenate([lat, np.full(P, 5.0),
                          (rng.integers(1, 11, P).astype(float) if integer else
                           rng.uniform(1, 10, P))])
    loss = np.concatenate([loss, np.zeros(P), rng.uniform(0, 0.01, P)])
    vloss = np.concatenate([np.zeros(R), rng.uniform(0, 0.05, P)])
    return (R + P, np.array(eu, np.int32), np.array(ev, np.int32), lat, loss, vloss)


def main():
    out = {}
    # 1. tcp test topologies (lossless / lossy) -- src/test/tcp/tcp-blocking-*.test.shadow.config.xml
    tcp = {}
    for name, loss in (("lossless", "0.0"), ("lossy", "0.25")):
        xml = TCP_GRAPHML % loss
        g = oracle.OGraph.from_graphml(xml.encode())
        lat, rel = g.complete_pairs([0], [0])
        tcp[name] = dict(graphml=xml, latency=float(lat[0]), reliability=float(rel[0]))
    assert tcp["lossless"]["latency"] == 50.0 and tcp["lossless"]["reliability"] == 1.0
    assert tcp["lossy"]["latency"] == 50.0 and tcp["lossy"]["reliability"] == 0.75
    json.dump(tcp, open(os.path.join(HERE, "tcp_1vertex.json"), "w"), indent=1)

    # 2. config 1: topology.simple, 2 hosts, seed chain from --seed 1
    g = oracle.OGraph.from_graphml(bundled("topology.simple"))
    master = 1
    slave_seed, master = oracle.rand_r(master)
    slave = slave_seed
    hosts = []
    for k in range(2):
        node_seed, slave = oracle.rand_r(slave)
        draw, _ = oracle.next_double(node_seed)
        v, st, _ = oracle.attach_vertex(g.vattrs, node_seed)
        hosts.append(dict(node_seed=node_seed, first_draw=draw, vertex=v,
                          vertex_id=g.vattrs["id"][v]))
    a, lat, rel, hops = g.table([h["vertex"] for h in hosts])
    json.dump(dict(slave_seed=slave_seed, hosts=hosts, attached=a.tolist(), lat=lat.tolist(),
                   rel=rel.tolist(), global_min=float(lat.min())),
              open(os.path.join(HERE, "c1_simple.json"), "w"), indent=1)

    # 3. configs 2 / 3: one host per vertex through its unique geocode
    tabs = {}
    rng = np.random.default_rng(2026)
    for name in ("topology", "topology.plab"):
        g = oracle.OGraph.from_graphml(bundled(name))
        st = 1
        verts = []
        for v in range(g.V):
            st = (st * 1103515245 + 12345) & 0xFFFFFFFF
            vv, _, _ = oracle.attach_vertex(g.vattrs, st, geocode_hint=g.vattrs["geocode"][v])
            verts.append(vv)
        a, lat, rel, hops = g.table(verts)
        k = rng.integers(0, len(a), (1000, 2))
        tabs[name] = dict(
            A=len(a), sha256_lat=hashlib.sha256(lat.tobytes()).hexdigest(),
            sha256_rel=hashlib.sha256(rel.tobytes()).hexdigest(), global_min=float(lat.min()),
            samples=[[int(i), int(j), float(lat[i, j]), float(rel[i, j])] for i, j in k])
    json.dump(tabs, open(os.path.join(HERE, "bundled_tables.json"), "w"), indent=1)

    # 4. synthetic non-complete graphs: 16 SSSP rows each
    for tag, integer in (("real", False), ("int", True)):
        V, eu, ev, elat, eloss, vloss = synth_graph(7 if integer else 8, 1400, 100, 11000,
                                                    integer)
        g = oracle.OGraph(V, eu, ev, elat, eloss, vloss)
        srcs = np.arange(1400, 1416, dtype=np.int32)
        targets = np.arange(1400, 1500, dtype=np.int32)
        lat, rel, hops = g.source_rows(srcs, targets)
        dists, parents, ties = [], [], []
        for s in srcs:
            d, pv, pe, _ = g.dijkstra(int(s))
            dists.append(d)
            parents.append(pv)
            ties.append(int((g.parent_ties(d, int(s)) >= 2).sum()))
        np.savez_compressed(os.path.join(HERE, "synth_%s.npz" % tag), V=V, eu=eu, ev=ev,
                            elat=elat, eloss=eloss, vloss=vloss, sources=srcs, targets=targets,
                            lat=lat, rel=rel, hops=hops, dist=np.array(dists),
                            parent=np.array(parents), tied_vertices=np.array(ties))

    # 5. packet routes
    rng = np.random.default_rng(11)
    n = 1000
    lat = rng.uniform(1, 300, n)
    lat[:10] = [1.0, 0.5, 1e-7, 123.456789, 50.0, 0.000001, 1e3, 2.5e-6, 7.0, 99.999999]
    rel = np.where(rng.random(n) < 0.1, 1.0, rng.uniform(0.5, 1.0, n))
    rel[10:20] = 0.0
    payload = np.where(rng.random(n) < 0.8, 1448, 0).astype(np.uint32)
    state = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    now = rng.integers(0, 10**12, n).astype(np.uint64)
    jump = 7_000_000
    t_c, d_c, s_c = oracle.route_packets(lat, rel, payload, state, now, jump, 1)
    t_n, d_n, s_n = oracle.route_packets(lat, rel, payload, state, now, jump, 0)
    np.savez_compressed(os.path.join(HERE, "packets.npz"), lat=lat, rel=rel, payload=payload,
                        state=state, now=now, jump=jump, time_clamp=t_c, delivered=d_c,
                        state_out=s_c, time_noclamp=t_n)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
