"""fleet.base.util_factory (reference: .../fleet/base/util_factory.py)."""
from .. import UtilBase  # noqa: F401
