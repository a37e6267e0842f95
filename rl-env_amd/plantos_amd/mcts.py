"""Batched MCTS: the reference's MCTS.search for every env of a batch at once.

Mirrors mcts_custom_trainer.MCTS (mcts_custom_trainer.py:72-243): same constructor
arguments and defaults (n_simulations=100, c_param=1.414, max_depth=50), same
search semantics bit for bit (UCB1 selection, random expansion, 70/30
least-visited-neighbour rollouts, +500 for a rollout that ends fully explored,
best_action by mean value), each env with its own np.random stream (numpy legacy
RandomState; env e starts as np.random.seed(seed + e)).  The whole search runs in
the HIP kernels of libplantos_hip.so (pe_mcts_*); it reads the live batch state
and modifies nothing -- step the chosen actions with the batch as usual.

    mcts = MCTS(vec_env, n_simulations=50, max_depth=100)   # train_mcts (:275)
    actions = mcts.search()                                  # int32 [N], device
    vec_env.step(actions)
"""
import ctypes

import numpy as np
import torch

from . import _capi as C
from .batch import PlantOSBatch


def _vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class MCTS:
    def __init__(self, env, n_simulations=100, c_param=1.414, max_depth=50, seed=0):
        self.batch = env if isinstance(env, PlantOSBatch) else env.batch
        self.n_simulations = int(n_simulations)
        self.c_param = float(c_param)
        self.max_depth = int(max_depth)
        self.num_envs = self.batch.num_envs
        h = ctypes.c_void_p()
        C.check(C.lib().pe_mcts_create(self.batch.handle, self.n_simulations, self.c_param, self.max_depth,
                                       ctypes.byref(h)), "pe_mcts_create")
        self._h = h
        dev = self.batch.device
        n = self.num_envs
        self.actions = torch.zeros(n, dtype=torch.int32, device=dev)
        self.root_order = torch.full((n, 5), -1, dtype=torch.int32, device=dev)
        self.root_visits = torch.zeros((n, 5), dtype=torch.int32, device=dev)
        self.root_value = torch.zeros((n, 5), dtype=torch.float64, device=dev)
        self.seed(seed)

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.batch.device).cuda_stream)

    def seed(self, seed=0):
        """np.random.seed(...) per env: an int gives env e the seed `seed + e`; a
        sequence gives every env its own seed."""
        if np.ndim(seed) == 0:
            C.check(C.lib().pe_mcts_seed(self._h, None, int(seed) & 0xFFFFFFFF, self._stream()), "pe_mcts_seed")
        else:
            s = np.ascontiguousarray(seed, np.uint32)
            if s.shape != (self.num_envs,):
                raise ValueError(f"expected {self.num_envs} seeds")
            C.check(C.lib().pe_mcts_seed(self._h, s.ctypes.data_as(ctypes.c_void_p), 0, self._stream()),
                    "pe_mcts_seed")

    def set_rng_state(self, key, pos):
        """key uint32 [N, 624], pos int [N]: numpy's get_state()[1], [2] per env."""
        key = np.ascontiguousarray(key, np.uint32).reshape(self.num_envs, 624)
        pos = np.ascontiguousarray(pos, np.int32).reshape(self.num_envs)
        C.check(C.lib().pe_mcts_set_rng(self._h, key.ctypes.data_as(ctypes.c_void_p),
                                        pos.ctypes.data_as(ctypes.c_void_p)), "pe_mcts_set_rng")

    def get_rng_state(self):
        key = np.zeros((self.num_envs, 624), np.uint32)
        pos = np.zeros(self.num_envs, np.int32)
        C.check(C.lib().pe_mcts_get_rng(self._h, key.ctypes.data_as(ctypes.c_void_p),
                                        pos.ctypes.data_as(ctypes.c_void_p)), "pe_mcts_get_rng")
        return key, pos

    def search(self, initial_state=None, mask=None, root_stats=False):
        """One MCTS.search per env (masked envs only, if `mask` is given).  The
        reference's `initial_state` observation is accepted and unused, as there.
        Returns the device int32 action tensor (or, with root_stats=True, also the
        root children: order [N,5] (-1 pad), visits [N,5], value f64 [N,5])."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.batch.device).to(torch.uint8).contiguous()
        rs = (self.root_order, self.root_visits, self.root_value) if root_stats else (None, None, None)
        C.check(C.lib().pe_mcts_search(self._h, _vp(m), _vp(self.actions), _vp(rs[0]), _vp(rs[1]), _vp(rs[2]),
                                       self._stream()), "pe_mcts_search")
        if root_stats:
            return self.actions, self.root_order, self.root_visits, self.root_value
        return self.actions

    def close(self):
        if getattr(self, "_h", None):
            C.check(C.lib().pe_mcts_destroy(self._h), "pe_mcts_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
