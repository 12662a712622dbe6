"""The source grouping's forest preorder (HostPrep::tree_order, topo_internal.h; round 6): equal
to the lexicographic order of the root-first h0-tree parent paths the grouping sorted by before,
with each vertex's depth, on random forests (host code: tests/c/tree_order_check.cpp, built by
the library's Makefile)."""
import os
import subprocess

from conftest import ROOT


def test_tree_order_equals_path_order():
    exe = os.path.join(ROOT, "tests", "c", "tree_order_check")
    assert os.path.exists(exe), "built by make -C shadow_amd/csrc"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
