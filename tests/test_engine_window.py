"""Engine-side window adapter through the C ABI, as Shadow would link it.

tests/c/engine_window.c emulates Shadow's worker around the product adapter of
include/shd_topology_window.h: hosts with their own rand_r streams (seed
chain of shd-master.c / shd-create-node.c), attach through topology_attach, packets emitted in
windows with other draws interleaved on the sender's stream.  The per-packet reference sequence
(getReliability, random_nextDouble, getLatency, clamp: shd-worker.c:332-370) runs on a twin
topology; the adapter captures the pre-draw state, advances the stream, and routes the whole
window with topology_routePacketBatch.  Delivered flags, delivery times, post-draw states,
every host stream and the lazily materialised minimum must be identical.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c", "engine_window")


def test_engine_window_binary_built_and_linked():
    """build() links the adapter test against the product library (no GPU needed to check)."""
    assert os.path.exists(BIN), "run __graft_entry__.build() (make -C shadow_amd/csrc)"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libshdtopo.so" in out and "libshdtopo_shim.so" in out
    assert "liboracle" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("serial", [0, 1])
def test_engine_window_batch_equals_per_packet_reference(serial):
    """The product adapter (topowindow_emit / topowindow_flush) against the per-packet getters:
    multi-threaded windows (runahead jump, clamp) and serial-mode windows (no clamp; every
    arrival lands at or after the window end, so deferring the routes changes no time)."""
    r = subprocess.run([BIN, "4", "20000", str(serial)], capture_output=True, text=True,
                       timeout=240)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "0 mismatches" in r.stdout
