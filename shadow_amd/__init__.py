"""shadow_amd -- MI355X-native routing engine for Shadow's topology subsystem.

The product is ``libshdtopo.so`` (HIP kernels for gfx950 + C++ host runtime) behind the C ABI
in ``include/shd_topology_abi.h``; this package is the Python mirror of the reference's
topology interface (``topology.py``) and the one-process-per-GPU sharding driver
(``sharding.py``).  See DESIGN.md.
"""
from .topology import Address, Random, Topology, ip_to_network, network_to_ip  # noqa: F401

__all__ = ["Address", "Random", "Topology", "ip_to_network", "network_to_ip"]
