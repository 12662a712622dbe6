"""ctypes binding of libshdtopo.so (include/shd_topology_abi.h).

The shared objects are built in-tree by ``make -C shadow_amd/csrc`` (``__graft_entry__.build``).
There is no fallback: if the library is missing, importing the product raises.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SHDTOPO_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("SHDTOPO_LIB") or os.path.join(HERE, "libshdtopo.so")
SHIM_PATH = os.path.join(HERE, "libshdtopo_shim.so")

P = ctypes.c_void_p
i32, i64, u32, u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64
dbl = ctypes.c_double
cstr = ctypes.c_char_p


class TopoPacketIn(ctypes.Structure):
    _fields_ = [("srcIP", u32), ("dstIP", u32), ("payloadLength", u32), ("rngState", u32),
                ("now", u64)]


class TopoPacketOut(ctypes.Structure):
    _fields_ = [("time", u64), ("rngState", u32), ("delivered", ctypes.c_uint8),
                ("_pad", ctypes.c_uint8 * 3)]


class ShdStats(ctypes.Structure):
    _fields_ = [("build_ms", dbl), ("sssp_kernel_ms", dbl), ("route_kernel_ms", dbl),
                ("sources", i64), ("targets", i64), ("ambiguous_pairs", i64),
                ("relaxations", i64), ("long_paths", i64), ("errors", i64),
                ("phase_ms", dbl * 4), ("near_iterations", i64), ("far_splits", i64),
                ("slots", i64), ("events", i64 * 8), ("far_scan_sources", i64), ("split_ms", dbl),
                ("batch", i64), ("lds_hubs", i64), ("replay_rows", i64), ("replay_ms", dbl),
                ("replay_pops", i64), ("replay_pushes", i64), ("replay_modifies", i64),
                ("replay_slots", i64), ("route_bad_packets", i64), ("devices", i64),
                ("exchange_ms", dbl), ("parent_phase_ms", dbl * 4), ("replay_lines", i64 * 6), ("batch_fill", i64), ("replay_phase_ms", dbl * 4),
                ("replay_sink_rounds", i64), ("replay_heap_sum", i64),
                ("replay_sink_ms", dbl * 3), ("replay_pf_hits", i64),
                ("replay_skips", i64), ("tie_dense", i64),
                ("batch_wave_ms", dbl * 6), ("batch_rounds", i64), ("batch_edges_b", i64),
                ("target_kappa_iters", i64), ("target_prep_ms", dbl),
                ("csr_ms", dbl), ("csr_host_ms", dbl), ("csr_copy_ms", dbl), ("csr_h0_rounds", i64),
                ("order_ms", dbl),
                ("replay_prep_ms", dbl), ("touched_lines", i64), ("csr_host_runs", i64),
                ("workspace_ms", dbl), ("csr_step_ms", dbl * 8), ("module_load_ms", dbl),
                ("build_wall_ms", dbl), ("walk_steps", i64), ("build_step_ms", dbl * 8),
                ("exchange_kind", i64), ("walk_kinds", i64 * 4),
                ("build_wait_ms", dbl), ("attach_prep_ms", dbl), ("replay_int_keys", i64),
                ("tie_probe_rows", i64), ("tie_probe_flagged", i64), ("tie_probe_ms", dbl),
                ("first_attach_to_table_ms", dbl), ("exchange_bytes", i64),
                ("csr_host_runs_total", i64), ("sweep_events", i64 * 4),
                ("write_lines", i64 * 16), ("read_lines", i64 * 8),
                ("attach_prep_step_ms", dbl * 4), ("pair_matrix_builds", i64),
                ("device_kernel_ms", dbl * 8), ("device_build_ms", dbl * 8),
                ("device_rows", i64 * 8), ("dev_inits", i64), ("init_bg_ms", dbl),
                ("path_seconds_total", dbl), ("paths_computed", i64),
                ("batch_layout_measured", i64), ("batches", i64), ("rows_to_host", i64),
                ("rows_to_host_ms", dbl), ("prep_trigger", i64),
                ("exchange_exposed_ms", dbl), ("workspace_bytes", i64)]


class ShdSynthParams(ctypes.Structure):
    _fields_ = [("seed", u64), ("n_routers", i64), ("n_poi", i64), ("n_edges", i64),
                ("integer_latency", ctypes.c_int), ("alpha", dbl), ("directed", ctypes.c_int)]


# every symbol include/shd_topology_abi.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "topology_new": (P, [cstr]),
    "topology_free": (None, [P]),
    "topology_attach": (None, [P, P, P, cstr, cstr, cstr, P, P]),
    "topology_detach": (None, [P, P]),
    "topology_isRoutable": (ctypes.c_int, [P, P, P]),
    "topology_getLatency": (dbl, [P, P, P]),
    "topology_getReliability": (dbl, [P, P, P]),
    "topology_getMinimumLatency": (dbl, [P]),
    "topology_routePacketBatch": (ctypes.c_int, [P, P, P, ctypes.c_size_t, u64, ctypes.c_int]),
    "shdtopo_version": (ctypes.c_int, []),
    "shdtopo_new_from_buffer": (P, [cstr, ctypes.c_size_t]),
    "shdtopo_set_option": (ctypes.c_int, [P, cstr, dbl]),
    "shdtopo_attach_ip": (i32, [P, u32, P, cstr, cstr, cstr, P, P]),
    "shdtopo_detach_ip": (None, [P, u32]),
    "shdtopo_get_latency_ip": (dbl, [P, u32, u32]),
    "shdtopo_get_reliability_ip": (dbl, [P, u32, u32]),
    "shdtopo_num_vertices": (i64, [P]),
    "shdtopo_num_edges": (i64, [P]),
    "shdtopo_is_complete": (ctypes.c_int, [P]),
    "shdtopo_is_directed": (ctypes.c_int, [P]),
    "shdtopo_num_attached": (i64, [P]),
    "shdtopo_attached_vertices": (i64, [P, P, i64]),
    "shdtopo_column_of_ip": (i32, [P, u32]),
    "shdtopo_vertex_of_ip": (i32, [P, u32]),
    "shdtopo_build": (ctypes.c_int, [P]),
    "shdtopo_shard_rows": (None, [i64, ctypes.c_int, ctypes.c_int, P, P]),
    "shdtopo_build_rows": (ctypes.c_int, [P, i64, i64, P, P, P, P]),
    "shdtopo_bind_table": (ctypes.c_int, [P, P, P, dbl, P]),
    "shdtopo_bind_table_ref": (ctypes.c_int, [P, P, P, dbl, P]),
    "shdtopo_rebuild": (ctypes.c_int, [P]),
    "shdtopo_table_to_host": (ctypes.c_int, [P, P, P, P]),
    "shdtopo_route_batch_device": (ctypes.c_int, [P, P, P, P, P, P, i64, u64, ctypes.c_int, P,
                                                  P, P, P]),
    "shdtopo_route_batch_device_slot": (ctypes.c_int, [P, ctypes.c_int, P, P, P, P, P, i64, u64,
                                                       ctypes.c_int, P, P, P, P]),
    "shdtopo_window_hold": (ctypes.c_int, [P, ctypes.c_int]),
    "shdtopo_window_release": (ctypes.c_int, [P]),
    "shdtopo_route_batch_vertices": (ctypes.c_int, [P, P, P, P, P, P, ctypes.c_size_t, u64,
                                                    ctypes.c_int, P]),
    "shdtopo_get_lazy_minimum_latency": (dbl, [P]),
    "shdtopo_lazy_rows": (i64, [P, P, P, P, i64]),
    "shdtopo_get_stats": (ctypes.c_int, [P, P]),
    "shdtopo_write_graphml": (ctypes.c_int, [P, cstr]),
    "shdtopo_replay_source": (ctypes.c_int, [P, i32, ctypes.c_int, P, P]),
    "shdtopo_test_segsort": (ctypes.c_int, [P, i64, P, i64, ctypes.c_int, P, P]),
    "shdtopo_test_batch_layout": (ctypes.c_int, [P, i64, dbl, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, P, P, P]),
    "shdtopo_export_graph": (ctypes.c_int, [P, P, P, P, P, P]),
    "shdtopo_export_csr": (i64, [P, P, P, P, P, P]),
    "shdtopo_new_synthetic": (P, [P]),
    "shdtopo_synth_packets": (ctypes.c_int, [P, u64, i64, i64, u64, u64, P, P, P, P, P, P, P]),
}

# include/shd_topology_window.h
WINDOW_DELIVER = ctypes.CFUNCTYPE(None, P, P, ctypes.c_int, u64)
SIGNATURES.update({
    "topowindow_new": (P, [P]),
    "topowindow_free": (None, [P]),
    "topowindow_emit": (i64, [P, P, P, u32, P, u64, P]),
    "topowindow_emit_state": (i64, [P, u32, u32, u32, u32, u64, P]),
    "topowindow_pending": (i64, [P]),
    "topowindow_flush": (ctypes.c_int, [P, u64, ctypes.c_int, WINDOW_DELIVER, P]),
    "topowindow_jump_ns": (u64, [P, u64]),
    "topowindow_serial_window_ns": (u64, [P]),
})

SHIM_SIGNATURES = {
    "shim_address_new": (P, [u32]),
    "shim_address_free": (None, [P]),
    "address_toNetworkIP": (u32, [P]),
    "random_new": (P, [ctypes.c_uint]),
    "random_free": (None, [P]),
    "random_nextDouble": (dbl, [P]),
    "random_nextInt": (ctypes.c_int, [P]),
    "shim_random_state": (ctypes.c_uint, [P]),
    "worker_updateMinTimeJump": (None, [dbl]),
    "shim_last_min_latency": (dbl, []),
    "shim_next_min_jump": (u64, []),
    "shim_min_updates": (ctypes.c_int, []),
    "shim_reset": (None, []),
    "logging_log": (None, [cstr, ctypes.c_int, cstr, cstr, ctypes.c_int, cstr]),
    "shim_log_count": (ctypes.c_int, []),
    "shim_log_criticals": (ctypes.c_int, []),
    "shim_log_get": (ctypes.c_int, [ctypes.c_int, P, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.c_char_p, ctypes.c_int]),
    "shim_log_reset": (None, []),
}

_lib = None
_shim = None


class LibraryMissing(RuntimeError):
    pass


def _bind(L, sigs, optional=False):
    for name, (res, args) in sigs.items():
        if optional and not hasattr(L, name):
            continue  # an A/B build of an older revision (SHDTOPO_LIB) lacks newer entry points
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def load():
    """Load the shim (RTLD_GLOBAL, so libshdtopo's weak Shadow imports resolve) and the engine."""
    global _lib, _shim
    if _lib is not None:
        return _lib, _shim
    for p in (SHIM_PATH, LIB_PATH):
        if not os.path.exists(p):
            raise LibraryMissing(
                "%s is not built: run `make -C shadow_amd/csrc` (or __graft_entry__.build()); "
                "the routing engine has no CPU fallback" % p)
    _shim = ctypes.CDLL(SHIM_PATH, mode=ctypes.RTLD_GLOBAL)
    _bind(_shim, SHIM_SIGNATURES)
    _lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    _bind(_lib, SIGNATURES, optional=bool(os.environ.get("SHDTOPO_LIB")))
    return _lib, _shim
