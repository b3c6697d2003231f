"""``fluid.incubate.data_generator`` (reference: fluid/incubate/data_generator)."""
from ...parallel.fleet.data_generator import *  # noqa: F401,F403
from ...parallel.fleet.data_generator import MultiSlotDataGenerator, MultiSlotStringDataGenerator  # noqa: F401
