"""Network topology (rack awareness) for locality-aware map placement."""
from .topology import DEFAULT_RACK, Topology

__all__ = ["DEFAULT_RACK", "Topology"]
