"""The drop-in getters under Shadow's threading contract.

tests/c/getters_mt.c links libshdtopo.so + libshdtopo_shim.so as Shadow would and runs 16 worker
threads on topology_getReliability / topology_getLatency / topology_isRoutable
(src/engine/shd-worker.c:179-203,352-360) of a lazy-mode, non-complete topology of 3,000
vertices from before its first table exists, with a late attach of hosts on new vertices under
them.  Every answer must be T[s][d] or T[d][s] of the final table bit for bit, the lazy running
minimum must equal the minimum over the materialised rows (exactly at a quiescent point, and
through the offered row minima at the end), getMinimumLatency the table minimum, and no critical
line may be logged.  Integer latencies (heavy ties: rows through the heap replay) and real ones.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "getters_mt")


def test_getters_mt_binary_built_and_linked():
    assert os.path.exists(BIN), "run __graft_entry__.build() (make -C shadow_amd/csrc)"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libshdtopo.so" in out and "libshdtopo_shim.so" in out
    assert "liboracle" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("integer", [0, 1])
def test_getters_concurrent_with_late_attach(integer):
    r = subprocess.run([BIN, str(integer), "16", "20000"], capture_output=True, text=True,
                       timeout=110)
    print(r.stdout, r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "0 mismatches" in r.stdout
    # rows copied one at a time on first read, never the whole table
    assert "rows copied to the host" in r.stdout
