"""The target-aware re-sort's segmented sort (topo_sssp_batch.hip: rows of <= 64 keys by waves,
<= 4,096 by workgroups in LDS, longer rows by hipcub) against the whole-adjacency hipcub
segmented radix sort it replaced and against numpy's stable argsort: the same keys and the same
positions, bit for bit (ties keep row order; -0.0 and +0.0 are equal keys, as in hipcub)."""
import numpy as np
import pytest

from shadow_amd import _lib


def _segsort(rowptr, keys, reference):
    lib, _ = _lib.load()
    rowptr = np.ascontiguousarray(rowptr, dtype=np.uint32)
    keys = np.ascontiguousarray(keys, dtype=np.float32)
    out_k = np.empty_like(keys)
    out_i = np.empty(len(keys), np.uint32)
    r = lib.shdtopo_test_segsort(rowptr.ctypes.data, len(rowptr) - 1, keys.ctypes.data, len(keys),
                                 1 if reference else 0, out_k.ctypes.data, out_i.ctypes.data)
    assert r == 0
    return out_k, out_i


def _expected(rowptr, keys):
    idx = np.empty(len(keys), np.uint32)
    for b, e in zip(rowptr[:-1], rowptr[1:]):
        idx[b:e] = b + np.argsort(keys[b:e], kind="stable")
    return keys[idx], idx


@pytest.mark.gpu
@pytest.mark.parametrize("ties", [False, True])
def test_segmented_sort_equals_hipcub_and_numpy(ties):
    rng = np.random.default_rng(7 if ties else 8)
    # every size class and its edges, between many short rows (the bulk of a power-law graph)
    edges = [0, 1, 2, 3, 63, 64, 65, 100, 127, 128, 129, 1000, 2048, 4095, 4096, 4097, 5000, 20000]
    lens = list(rng.integers(0, 40, 3000)) + edges + list(rng.integers(0, 40, 500)) + edges[::-1]
    rowptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
    n = int(rowptr[-1])
    if ties:
        pool = np.array([-np.inf, -3.5, -0.0, 0.0, 1e-30, 0.25, 0.25, 7.0, 1e30, np.inf], np.float32)
        keys = pool[rng.integers(0, len(pool), n)]
    else:
        keys = (rng.standard_normal(n) * 100).astype(np.float32)
        keys[rng.integers(0, n, 200)] = -0.0
        keys[rng.integers(0, n, 200)] = 0.0
        keys[rng.integers(0, n, 50)] = np.inf
        keys[rng.integers(0, n, 50)] = -np.inf
    k_new, i_new = _segsort(rowptr, keys, reference=False)
    k_ref, i_ref = _segsort(rowptr, keys, reference=True)
    k_np, i_np = _expected(rowptr, keys)
    assert np.array_equal(i_new, i_ref)
    assert np.array_equal(k_new.view(np.uint32), k_ref.view(np.uint32))
    assert np.array_equal(i_new, i_np)
    assert np.array_equal(k_new.view(np.uint32), k_np.view(np.uint32))


def test_segmented_sort_rejects_bad_offsets():
    """Argument checks run before any device use (CPU)."""
    lib, _ = _lib.load()
    keys = np.zeros(4, np.float32)
    out_k = np.empty(4, np.float32)
    out_i = np.empty(4, np.uint32)
    for rp in ([0, 3, 2, 4], [1, 2, 4], [0, 2, 5]):
        rp = np.array(rp, np.uint32)
        assert lib.shdtopo_test_segsort(rp.ctypes.data, len(rp) - 1, keys.ctypes.data, 4, 0,
                                        out_k.ctypes.data, out_i.ctypes.data) == -1
