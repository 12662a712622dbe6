import lzma
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_RESOURCE = "/root/reference/resource"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


def bundled_topology(name):
    """Bundled topology XML bytes.  The GPU box has no /root/reference, so the three bundled
    files are vendored as data fixtures (xz, byte-identical) under tests/golden/resource/."""
    p = os.path.join(GOLDEN, "resource", name + ".graphml.xml.xz")
    if not os.path.exists(p):
        p = os.path.join(REF_RESOURCE, name + ".graphml.xml.xz")
    with lzma.open(p) as f:
        return f.read()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
