"""``fleet.data_generator`` (reference: python/paddle/distributed/fleet/data_generator)."""
from .. import MultiSlotDataGenerator, MultiSlotStringDataGenerator  # noqa: F401

DataGenerator = MultiSlotDataGenerator
__all__ = ["DataGenerator", "MultiSlotDataGenerator", "MultiSlotStringDataGenerator"]
