"""``paddle.profiler.profiler`` module path (the Profiler of paddle.profiler)."""
from . import *  # noqa: F401,F403
from . import Profiler, ProfilerState, ProfilerTarget, make_scheduler, export_chrome_tracing  # noqa: F401
