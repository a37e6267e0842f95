"""Minimal gymnasium.spaces stand-in (Discrete, Box) for tools/gen_golden.py."""
import numpy as np


class Discrete:
    def __init__(self, n):
        self.n = int(n)

    def contains(self, x):
        return 0 <= int(x) < self.n


class Box:
    def __init__(self, low, high, shape, dtype):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)
