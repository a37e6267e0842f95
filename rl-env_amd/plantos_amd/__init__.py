"""plantos_amd -- MI355X-native batched PlantOSEnv (GammaKing2000/RL-Env hot path).

Public surface:
  PlantOSBatch      N envs in HBM, device tensors in/out (C-ABI: include/plantos_batch.h)
  PlantOSVecEnv     Stable-Baselines3 VecEnv drop-in for DummyVecEnv (A2C_training.py:216-218)
  PlantOSVectorEnv  gymnasium-0.29 VectorEnv convention over the same batch
"""
from .batch import PlantOSBatch  # noqa: F401
from .vec_env import PlantOSVecEnv, PlantOSVectorEnv  # noqa: F401

__all__ = ["PlantOSBatch", "PlantOSVecEnv", "PlantOSVectorEnv"]
