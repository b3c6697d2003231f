"""``fleet.runtime`` (reference: python/paddle/distributed/fleet/runtime): the parameter-server
runtime of this framework (parallel/ps: the native table server and its client)."""
from ...ps import *  # noqa: F401,F403
