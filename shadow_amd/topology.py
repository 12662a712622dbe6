"""Python mirror of Shadow's topology interface (src/topology/shd-topology.h:14-22) over the
MI355X engine in libshdtopo.so.

Method names, argument meaning and error behaviour follow the reference:

* ``Topology.new(path)``            topology_new            (shd-topology.c:1237) -- None on failure
* ``attach(address, random, ...)``  topology_attach         (shd-topology.c:1154) -- one
                                    random_nextDouble draw on the host stream unless LPM
* ``detach(address)``               topology_detach         (shd-topology.c:1190)
* ``getLatency / getReliability``   (shd-topology.c:940-958) -- -1.0 for an unattached address
* ``isRoutable``                    (shd-topology.c:960)
* ``getMinimumLatency``             new: global min over attached pairs
* ``routePacketBatch``              new: worker_schedulePacket for a window (shd-worker.c:332-370)

``Address`` / ``Random`` are the shim restatements of Shadow's objects (libshdtopo_shim.so) so
that the exact C entry points are exercised.  Every computation runs in the HIP library; this
module only marshals arguments.
"""
from __future__ import annotations

import ctypes
import socket
import struct

import numpy as np

from . import _lib as L


def ip_to_network(ip: str) -> int:
    """dotted quad -> in_addr_t as Shadow holds it (network byte order in memory)."""
    return struct.unpack("<I", socket.inet_aton(ip))[0]


def network_to_ip(n: int) -> str:
    return socket.inet_ntoa(struct.pack("<I", n & 0xFFFFFFFF))


class Address:
    """Shadow Address (shd-address.c): only the network-order IP is used by the topology."""

    def __init__(self, ip):
        lib, shim = L.load()
        self.ip = ip_to_network(ip) if isinstance(ip, str) else int(ip)
        self._p = shim.shim_address_new(self.ip)
        self._shim = shim

    def __del__(self):
        try:
            self._shim.shim_address_free(self._p)
        except Exception:
            pass


class Random:
    """Shadow Random (shd-random.c): glibc rand_r stream."""

    def __init__(self, seed: int):
        lib, shim = L.load()
        self._p = shim.random_new(seed & 0xFFFFFFFF)
        self._shim = shim

    @property
    def state(self) -> int:
        return int(self._shim.shim_random_state(self._p))

    def nextDouble(self) -> float:
        return float(self._shim.random_nextDouble(self._p))

    def nextInt(self) -> int:
        return int(self._shim.random_nextInt(self._p))

    def __del__(self):
        try:
            self._shim.random_free(self._p)
        except Exception:
            pass


def _b(s):
    return None if s is None else s.encode()


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Topology:
    def __init__(self, handle):
        self._lib, self._shim = L.load()
        self._h = handle

    # ---- construction ----
    @classmethod
    def new(cls, graph_path: str):
        lib, _ = L.load()
        h = lib.topology_new(graph_path.encode())
        return cls(h) if h else None

    @classmethod
    def from_buffer(cls, graphml: bytes):
        lib, _ = L.load()
        h = lib.shdtopo_new_from_buffer(graphml, len(graphml))
        return cls(h) if h else None

    @classmethod
    def synthetic(cls, seed=20261015, n_routers=990_000, n_poi=10_000, n_edges=10_000_000,
                  integer_latency=False, alpha=1.0 / 1.1, directed=False):
        lib, _ = L.load()
        p = L.ShdSynthParams(seed, n_routers, n_poi, n_edges, int(integer_latency), alpha,
                             int(directed))
        h = lib.shdtopo_new_synthetic(ctypes.byref(p))
        return cls(h) if h else None

    def free(self):
        if self._h:
            self._lib.topology_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def set_option(self, key: str, value: float):
        if self._lib.shdtopo_set_option(self._h, key.encode(), float(value)) != 0:
            raise KeyError(key)

    # ---- reference API ----
    def attach(self, address: Address, random: Random, ipHint=None, geocodeHint=None,
               typeHint=None):
        down = ctypes.c_uint64(0)
        up = ctypes.c_uint64(0)
        self._lib.topology_attach(self._h, address._p, random._p, _b(ipHint), _b(geocodeHint),
                                  _b(typeHint), ctypes.byref(down), ctypes.byref(up))
        return down.value, up.value

    def detach(self, address: Address):
        self._lib.topology_detach(self._h, address._p)

    def isRoutable(self, src: Address, dst: Address) -> bool:
        return bool(self._lib.topology_isRoutable(self._h, src._p, dst._p))

    def getLatency(self, src: Address, dst: Address) -> float:
        return self._lib.topology_getLatency(self._h, src._p, dst._p)

    def getReliability(self, src: Address, dst: Address) -> float:
        return self._lib.topology_getReliability(self._h, src._p, dst._p)

    def getMinimumLatency(self) -> float:
        return self._lib.topology_getMinimumLatency(self._h)

    def lazyMinimumLatency(self) -> float:
        return self._lib.shdtopo_get_lazy_minimum_latency(self._h)

    def routePacketBatch(self, src_ip, dst_ip, payload, rng_state, now, jump_ns, clamp=True):
        n = len(src_ip)
        ins = (L.TopoPacketIn * n)()
        for i in range(n):
            ins[i].srcIP = int(src_ip[i])
            ins[i].dstIP = int(dst_ip[i])
            ins[i].payloadLength = int(payload[i])
            ins[i].rngState = int(rng_state[i])
            ins[i].now = int(now[i])
        outs = (L.TopoPacketOut * n)()
        r = self._lib.topology_routePacketBatch(self._h, ins, outs, n, int(jump_ns), int(clamp))
        if r < 0:
            raise RuntimeError("topology_routePacketBatch failed: %d" % r)
        self.last_unrouted = r  # packets whose address is not attached (delivered 0)
        t = np.array([o.time for o in outs], dtype=np.uint64)
        st = np.array([o.rngState for o in outs], dtype=np.uint32)
        dl = np.array([o.delivered for o in outs], dtype=np.uint8)
        return t, dl, st

    # ---- raw-IP helpers ----
    def attach_ip(self, ip, state, ipHint=None, geocodeHint=None, typeHint=None):
        st = ctypes.c_uint32(state & 0xFFFFFFFF)
        v = self._lib.shdtopo_attach_ip(self._h, int(ip), ctypes.byref(st), _b(ipHint),
                                        _b(geocodeHint), _b(typeHint), None, None)
        return v, st.value

    def detach_ip(self, ip):
        self._lib.shdtopo_detach_ip(self._h, int(ip))

    def latency_ip(self, s, d):
        return self._lib.shdtopo_get_latency_ip(self._h, int(s), int(d))

    def reliability_ip(self, s, d):
        return self._lib.shdtopo_get_reliability_ip(self._h, int(s), int(d))

    # ---- graph / table ----
    @property
    def num_vertices(self):
        return int(self._lib.shdtopo_num_vertices(self._h))

    @property
    def num_edges(self):
        return int(self._lib.shdtopo_num_edges(self._h))

    @property
    def is_complete(self):
        return bool(self._lib.shdtopo_is_complete(self._h))

    @property
    def is_directed(self):
        return bool(self._lib.shdtopo_is_directed(self._h))

    def attached_vertices(self):
        n = int(self._lib.shdtopo_num_attached(self._h))
        out = np.empty(max(n, 1), np.int32)
        self._lib.shdtopo_attached_vertices(self._h, _p(out), n)
        return out[:n]

    def vertex_of_ip(self, ip):
        return int(self._lib.shdtopo_vertex_of_ip(self._h, int(ip)))

    def lazy_rows(self):
        """Test hook (shdtopo_lazy_rows): the materialised source rows -- (vertices, epochs, the
        row minimum each latest materialisation offered to the running minimum)."""
        n = int(self._lib.shdtopo_lazy_rows(self._h, None, None, None, 0))
        v = np.empty(max(n, 1), np.int32)
        e = np.empty(max(n, 1), np.uint64)
        m = np.empty(max(n, 1), np.float64)
        n = int(self._lib.shdtopo_lazy_rows(self._h, _p(v), _p(e), _p(m), n))
        return v[:n], e[:n], m[:n]

    def column_of_ip(self, ip):
        return int(self._lib.shdtopo_column_of_ip(self._h, int(ip)))

    def build(self):
        r = self._lib.shdtopo_build(self._h)
        if r != 0:
            raise RuntimeError("shdtopo_build failed: %d" % r)

    def table(self):
        """Host copy of the A x A table: (attached vertices, lat, rel, hops)."""
        self.build()
        a = self.attached_vertices()
        n = len(a)
        lat = np.empty((n, n), np.float64)
        rel = np.empty((n, n), np.float64)
        hops = np.empty((n, n), np.uint16)
        r = self._lib.shdtopo_table_to_host(self._h, _p(lat), _p(rel), _p(hops))
        if r != 0:
            raise RuntimeError("shdtopo_table_to_host failed: %d" % r)
        return a, lat, rel, hops

    def stats(self):
        s = L.ShdStats()
        r = self._lib.shdtopo_get_stats(self._h, ctypes.byref(s))
        if r != 0:
            raise RuntimeError("shdtopo_get_stats failed: %d" % r)
        out = {k: getattr(s, k) for k, _ in L.ShdStats._fields_}
        out["phase_ms"] = list(out["phase_ms"])
        out["parent_phase_ms"] = list(out["parent_phase_ms"])
        out["replay_lines"] = list(out["replay_lines"])
        out["replay_phase_ms"] = list(out["replay_phase_ms"])
        out["replay_sink_ms"] = list(out["replay_sink_ms"])
        out["batch_wave_ms"] = list(out["batch_wave_ms"])
        out["csr_step_ms"] = list(out["csr_step_ms"])
        out["build_step_ms"] = list(out["build_step_ms"])
        out["walk_kinds"] = list(out["walk_kinds"])
        for k in ("device_kernel_ms", "device_build_ms", "device_rows", "attach_prep_step_ms",
                  "sweep_events", "write_lines", "read_lines"):
            out[k] = list(out[k])
        out["events"] = dict(zip(("expanded", "tail_relax", "tail_improve", "window_taken",
                                  "overflow_refilled", "parent_vertices", "tail_settled_relax",
                                  "stale_skipped"),
                                 list(out["events"])))
        return out

    def export_graph(self):
        """(V, eu, ev, elat, eloss, vloss) host arrays of the parsed graph (document order)."""
        V, E = self.num_vertices, self.num_edges
        eu = np.empty(E, np.int32)
        ev = np.empty(E, np.int32)
        el = np.empty(E, np.float64)
        lo = np.empty(E, np.float64)
        vl = np.empty(V, np.float64)
        if self._lib.shdtopo_export_graph(self._h, _p(eu), _p(ev), _p(el), _p(lo), _p(vl)) != 0:
            raise RuntimeError("export_graph failed")
        return V, eu, ev, el, lo, vl

    def export_csr(self):
        """Test hook (shdtopo_export_csr): the GPU-prepared CSR -- perm (new -> old), rowptr, the
        adjacency columns, pi = d(h0, .) and the h0-tree parents, relabelled ids."""
        n = int(self._lib.shdtopo_export_csr(self._h, None, None, None, None, None))
        if n < 0:
            raise RuntimeError("shdtopo_export_csr failed: %d" % n)
        V = self.num_vertices
        perm = np.empty(V, np.int32)
        rowptr = np.empty(V + 1, np.uint32)
        col = np.empty(max(n, 1), np.uint32)
        pot = np.empty(V, np.float64)
        par = np.empty(V, np.uint32)
        r = self._lib.shdtopo_export_csr(self._h, _p(perm), _p(rowptr), _p(col), _p(pot), _p(par))
        if r != n:
            raise RuntimeError("shdtopo_export_csr failed: %d" % r)
        return dict(perm=perm, rowptr=rowptr, col=col[:n], pot=pot, tree_parent=par)

    def replay_source(self, src, full=True):
        """Test hook (shdtopo_replay_source): the exact heap replay's (dist, parent vertex) from
        vertex `src`, original ids; full=False stops when every attached vertex is popped."""
        V = self.num_vertices
        dist = np.empty(V, np.float64)
        par = np.empty(V, np.int32)
        r = self._lib.shdtopo_replay_source(self._h, int(src), int(bool(full)), _p(dist), _p(par))
        if r != 0:
            raise RuntimeError("shdtopo_replay_source failed: %d" % r)
        return dist, par

    def write_graphml(self, path):
        if self._lib.shdtopo_write_graphml(self._h, path.encode()) != 0:
            raise RuntimeError("write_graphml failed")

    # ---- device-level boundary (torch tensors are used as plain HBM buffers) ----
    def build_rows_into(self, row0, row1, lr, hops, rowmin=None, stream=0):
        r = self._lib.shdtopo_build_rows(self._h, int(row0), int(row1), lr.data_ptr(),
                                         hops.data_ptr(),
                                         rowmin.data_ptr() if rowmin is not None else None,
                                         stream or None)
        if r != 0:
            raise RuntimeError("shdtopo_build_rows failed: %d" % r)

    def rebuild(self):
        """shdtopo_rebuild: build the whole table now (the getters build it lazily)."""
        r = self._lib.shdtopo_rebuild(self._h)
        if r != 0:
            raise RuntimeError("shdtopo_rebuild failed: %d" % r)

    def bind_table_ref(self, lr, hops, global_min, stream=0):
        """Install lr / hops in place (the tensors must outlive the binding)."""
        r = self._lib.shdtopo_bind_table_ref(self._h, lr.data_ptr(), hops.data_ptr(),
                                             float(global_min), stream or None)
        if r != 0:
            raise RuntimeError("shdtopo_bind_table_ref failed: %d" % r)
        self._bound = (lr, hops)  # keep the buffers alive while bound

    def bind_table(self, lr, hops, global_min, stream=0):
        r = self._lib.shdtopo_bind_table(self._h, lr.data_ptr(), hops.data_ptr(),
                                         float(global_min), stream or None)
        if r != 0:
            raise RuntimeError("shdtopo_bind_table failed: %d" % r)

    def route_batch_vertices(self, src_v, dst_v, payload, rng_state, now, jump_ns, clamp=True):
        """shdtopo_route_batch_vertices: (time, delivered, state, not-routed count)."""
        n = len(src_v)
        c = lambda x, t: np.ascontiguousarray(x, dtype=t)
        sv, dv = c(src_v, np.int32), c(dst_v, np.int32)
        pay, st, nw = c(payload, np.uint32), c(rng_state, np.uint32), c(now, np.uint64)
        outs = (L.TopoPacketOut * max(n, 1))()
        r = self._lib.shdtopo_route_batch_vertices(self._h, _p(sv), _p(dv), _p(pay), _p(st),
                                                   _p(nw), n, int(jump_ns), int(clamp), outs)
        if r < 0:
            raise RuntimeError("shdtopo_route_batch_vertices failed: %d" % r)
        t = np.array([outs[i].time for i in range(n)], dtype=np.uint64)
        s = np.array([outs[i].rngState for i in range(n)], dtype=np.uint32)
        dl = np.array([outs[i].delivered for i in range(n)], dtype=np.uint8)
        return t, dl, s, r

    def route_batch_device_slot(self, slot, src_col, dst_col, payload, state_in, now, jump_ns,
                                clamp, t_out, state_out, delivered, stream=0):
        r = self._lib.shdtopo_route_batch_device_slot(
            self._h, int(slot), src_col.data_ptr(), dst_col.data_ptr(), payload.data_ptr(),
            state_in.data_ptr(), now.data_ptr(), int(src_col.numel()), int(jump_ns), int(clamp),
            t_out.data_ptr(), state_out.data_ptr(), delivered.data_ptr(), stream or None)
        if r != 0:
            raise RuntimeError("shdtopo_route_batch_device_slot failed: %d" % r)

    def route_batch_device(self, src_col, dst_col, payload, state_in, now, jump_ns, clamp,
                           t_out, state_out, delivered, stream=0):
        r = self._lib.shdtopo_route_batch_device(
            self._h, src_col.data_ptr(), dst_col.data_ptr(), payload.data_ptr(),
            state_in.data_ptr(), now.data_ptr(), int(src_col.numel()), int(jump_ns), int(clamp),
            t_out.data_ptr(), state_out.data_ptr(), delivered.data_ptr(), stream or None)
        if r != 0:
            raise RuntimeError("shdtopo_route_batch_device failed: %d" % r)

    def synth_packets(self, seed, n_hosts, n_packets, t0, jump):
        """C5 workload: attach n_hosts Tor-like hosts and emit one window of packets."""
        n = int(n_packets)
        out = dict(src_col=np.empty(n, np.int32), dst_col=np.empty(n, np.int32),
                   payload=np.empty(n, np.uint32), state_in=np.empty(n, np.uint32),
                   now=np.empty(n, np.uint64), src_ip=np.empty(n, np.uint32),
                   dst_ip=np.empty(n, np.uint32))
        r = self._lib.shdtopo_synth_packets(
            self._h, int(seed), int(n_hosts), n, int(t0), int(jump), _p(out["src_col"]),
            _p(out["dst_col"]), _p(out["payload"]), _p(out["state_in"]), _p(out["now"]),
            _p(out["src_ip"]), _p(out["dst_ip"]))
        if r != 0:
            raise RuntimeError("shdtopo_synth_packets failed: %d" % r)
        return out


def shim():
    return L.load()[1]
