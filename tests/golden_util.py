"""Helpers to load the reference-generated fixtures (tests/golden/, tools/gen_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

INJECT_CFGS = ["g20", "g21", "g25", "g64", "g64r32", "g7", "g32"]
MAP_CFGS = ["g20", "g21", "g25", "g64", "g7", "g32"]
TRAJ_FILES = ["traj_g20_random", "traj_g20_explore", "traj_g7_explore", "traj_g21_explore"]


def load(name):
    """All arrays of one fixture, decompressed once (NpzFile re-reads per access)."""
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def cfg_tuple(f):
    G, P, O, R, C = (int(v) for v in f["config"])
    return G, P, O, R, C
