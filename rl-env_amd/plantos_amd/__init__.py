"""plantos_amd -- MI355X-native batched PlantOSEnv (GammaKing2000/RL-Env hot path).

Public surface:
  PlantOSBatch   N envs in HBM, device tensors in/out (C-ABI: include/plantos_batch.h)
"""
from .batch import PlantOSBatch  # noqa: F401

__all__ = ["PlantOSBatch"]
