"""babble_amd — MI355X-native hashgraph consensus-ordering engine.

The hot path of mpitid/babble's `hashgraph` package (InsertEvent coordinates,
DivideRounds, DecideFame, FindOrder) as hand-written HIP kernels for gfx950
behind a C ABI (include/hge.h).  `babble_amd.engine.Engine` is the Python
front-end used by tests and bench.py; `babble_amd.gossip` generates the
seeded synthetic workloads.
"""
from . import gossip  # noqa: F401

__all__ = ["gossip", "engine"]
