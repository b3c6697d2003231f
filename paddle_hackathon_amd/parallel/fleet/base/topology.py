"""fleet.base.topology (reference: .../fleet/base/topology.py)."""
from ...topology import *  # noqa: F401,F403
