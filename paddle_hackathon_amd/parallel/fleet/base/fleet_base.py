"""fleet.base.fleet_base (reference: .../fleet/base/fleet_base.py)."""
from .. import Fleet  # noqa: F401
