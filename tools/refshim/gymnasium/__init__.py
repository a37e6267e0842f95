"""Minimal stand-in for gymnasium 0.29.1, used ONLY by tools/gen_golden.py.

gymnasium is not installed in this image (no network).  The reference's
step/reset math never touches gymnasium beyond these names
(SURVEY.md §8(c)); render paths are never exercised by the generator.
"""
import numpy as np

from . import spaces  # noqa: F401


class Env:
    def reset(self, seed=None, options=None):
        # gymnasium.Env.reset seeds self.np_random; plantos_env never uses it.
        self.np_random = np.random.default_rng(seed)
        return None


class Wrapper(Env):
    def __init__(self, env):
        self.env = env


def register(*args, **kwargs):
    return None
