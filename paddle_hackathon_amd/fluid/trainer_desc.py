"""``fluid.trainer_desc`` (reference python/paddle/fluid/trainer_desc.py): trainer configurations
run by static/trainer.py."""
from ..static.trainer import (TrainerDesc, MultiTrainer, DistMultiTrainer, PipelineTrainer, HeterXpuTrainer,  # noqa: F401
                              PSGPUTrainer, HeterPipelineTrainer)

__all__ = ["TrainerDesc", "MultiTrainer", "DistMultiTrainer", "PipelineTrainer", "HeterXpuTrainer", "PSGPUTrainer",
           "HeterPipelineTrainer"]
