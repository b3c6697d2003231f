"""fleet.base.role_maker (reference: python/paddle/distributed/fleet/base/role_maker.py)."""
from ..role_maker import *  # noqa: F401,F403
from ..role_maker import Role, PaddleCloudRoleMaker, UserDefinedRoleMaker  # noqa: F401
