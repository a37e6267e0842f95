"""ctypes wrapper of the C parity oracle (oracle/plantos_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package (rl-env_amd/).
The oracle restates /root/reference/plantos_env.py step/reset (file:line
citations in plantos_oracle.c) and is pinned against the reference's own
outputs in tests/golden/ (tests/test_oracle_golden.py).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libplantos_oracle.so")

NSCAL = 8
S_X, S_Y, S_STEP, S_COLL, S_COLLIDED, S_BONUS, S_POISONED, S_EPISODE = range(8)


class POConfig(ctypes.Structure):
    _fields_ = [
        ("grid_size", ctypes.c_int32), ("num_plants", ctypes.c_int32), ("num_obstacles", ctypes.c_int32),
        ("lidar_range", ctypes.c_int32), ("lidar_channels", ctypes.c_int32), ("max_steps", ctypes.c_int32),
        ("thirsty_plant_prob", ctypes.c_double),
        ("r_goal", ctypes.c_double), ("r_mistake", ctypes.c_double), ("r_invalid", ctypes.c_double),
        ("r_water_empty", ctypes.c_double), ("r_step", ctypes.c_double), ("r_exploration", ctypes.c_double),
        ("r_revisit", ctypes.c_double), ("r_complete", ctypes.c_double),
        ("map_algo", ctypes.c_int32), ("pad_", ctypes.c_int32),
    ]


class POMt(ctypes.Structure):
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("index", ctypes.c_int32)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        L.po_default_config.argtypes = [ctypes.POINTER(POConfig)] + [ctypes.c_int] * 5
        L.po_obs_dim.argtypes = [ctypes.POINTER(POConfig)]
        L.po_lidar_table.argtypes = [ctypes.c_int, ctypes.c_int, P, P]
        L.po_obs.argtypes = [ctypes.POINTER(POConfig), P, P, P, P]
        L.po_step_batch.argtypes = [ctypes.POINTER(POConfig), ctypes.c_int64, P, P, P, P, P, P, P, P, P]
        L.po_info.argtypes = [ctypes.POINTER(POConfig), P, P, P]
        L.po_reset_cpython.argtypes = [ctypes.POINTER(POConfig), ctypes.POINTER(POMt), P, P, P, P]
        L.po_reset_philox.argtypes = [ctypes.POINTER(POConfig), ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.c_uint32, P, P, P, P]
        L.po_mt_seed.argtypes = [ctypes.POINTER(POMt), ctypes.c_uint64]
        L.po_mt_u32.argtypes = [ctypes.POINTER(POMt)]
        L.po_mt_u32.restype = ctypes.c_uint32
        L.po_philox4x32.argtypes = [P, P, P]
        L.po_pyset_free_list.argtypes = [ctypes.c_int, P, P]
        L.po_bench.argtypes = [ctypes.POINTER(POConfig), ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                               ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        L.po_bench.restype = ctypes.c_double
        L.po_synth_action.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.po_synth_action.restype = ctypes.c_int32
        L.po_mt_seed_genrand.argtypes = [ctypes.POINTER(POMt), ctypes.c_uint32]
        L.po_np_random.argtypes = [ctypes.POINTER(POMt)]
        L.po_np_random.restype = ctypes.c_double
        L.po_np_randint.argtypes = [ctypes.POINTER(POMt), ctypes.c_int32]
        L.po_np_randint.restype = ctypes.c_int32
        L.po_mcts_search.argtypes = [ctypes.POINTER(POConfig), P, P, P, P, ctypes.POINTER(POMt), ctypes.c_int32,
                                     ctypes.c_double, ctypes.c_int32, P, P, P]
        L.po_mcts_search.restype = ctypes.c_int32
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def config(G, P, O, R, C, **overrides):
    c = POConfig()
    lib().po_default_config(ctypes.byref(c), G, P, O, R, C)
    for k, v in overrides.items():
        setattr(c, k, v)
    return c


def obs_dim(c):
    return 5 * c.lidar_channels + 27


def lidar_table(C, R):
    dx = np.zeros(C * R, np.int32)
    dy = np.zeros(C * R, np.int32)
    lib().po_lidar_table(C, R, _p(dx), _p(dy))
    return dx.reshape(C, R), dy.reshape(C, R)


class MT:
    """CPython `random` MT19937 stream (random.seed(int) semantics)."""

    def __init__(self, seed):
        self.s = POMt()
        lib().po_mt_seed(ctypes.byref(self.s), seed)

    def u32(self):
        return lib().po_mt_u32(ctypes.byref(self.s))


class NpMT:
    """numpy legacy RandomState stream (np.random.seed(int) semantics) on the oracle's MT."""

    def __init__(self, seed):
        self.s = POMt()
        lib().po_mt_seed_genrand(ctypes.byref(self.s), seed)

    def state(self):
        """(key uint32[624], pos) exactly as numpy's get_state() reports them."""
        return np.array(self.s.mt[:], np.uint32), int(self.s.index)

    def random(self):
        return lib().po_np_random(ctypes.byref(self.s))

    def randint(self, n):
        return lib().po_np_randint(ctypes.byref(self.s), n)


def mcts_search(cfg, cells, visits, explored, scal, rng, n_sims, c_param, max_depth):
    """MCTS.search (mcts_custom_trainer.py:91-139) of one env; rng (NpMT) advances.
    Returns (action, order[5], visits[5], value[5]) -- root children in insertion order."""
    cells = np.ascontiguousarray(cells, np.uint8)
    visits = np.ascontiguousarray(visits, np.int32)
    explored = np.ascontiguousarray(explored, np.int8)
    sc = np.zeros(NSCAL, np.int32)
    sc[:len(scal)] = scal
    order = np.zeros(5, np.int32)
    cv = np.zeros(5, np.int32)
    cval = np.zeros(5, np.float64)
    a = lib().po_mcts_search(ctypes.byref(cfg), _p(cells), _p(visits), _p(explored), _p(sc), ctypes.byref(rng.s),
                             n_sims, c_param, max_depth, _p(order), _p(cv), _p(cval))
    return a, order, cv, cval


class Batch:
    """n independent envs in the reference's own state terms (plantos_env.py:96-123)."""

    def __init__(self, cfg, n):
        self.cfg = cfg
        G = cfg.grid_size
        self.n = n
        self.cells = np.zeros((n, G, G), np.uint8)
        self.visits = np.zeros((n, G, G), np.int32)
        self.explored = np.zeros((n, G, G), np.int8)
        self.scal = np.zeros((n, NSCAL), np.int32)

    def _chk(self):
        for a in (self.cells, self.visits, self.explored, self.scal):
            assert a.flags.c_contiguous

    def step(self, actions):
        self._chk()
        a = np.ascontiguousarray(actions, np.int64)
        D = obs_dim(self.cfg)
        obs = np.zeros((self.n, D), np.float32)
        rew = np.zeros(self.n, np.float64)
        te = np.zeros(self.n, np.uint8)
        tr = np.zeros(self.n, np.uint8)
        lib().po_step_batch(ctypes.byref(self.cfg), self.n, _p(self.cells), _p(self.visits), _p(self.explored),
                            _p(self.scal), _p(a), _p(obs), _p(rew), _p(te), _p(tr))
        return obs, rew, te.astype(bool), tr.astype(bool)

    def obs(self, idx=None):
        self._chk()
        D = obs_dim(self.cfg)
        out = np.zeros((self.n, D), np.float32)
        for e in (range(self.n) if idx is None else idx):
            lib().po_obs(ctypes.byref(self.cfg), _p(self.cells[e]), _p(self.visits[e]), _p(self.scal[e]),
                         _p(out[e]))
        return out

    def info(self, e):
        out = np.zeros(5, np.int32)
        lib().po_info(ctypes.byref(self.cfg), _p(self.cells[e]), _p(self.explored[e]), _p(out))
        return out

    def reset_cpython(self, e, mt):
        rc = lib().po_reset_cpython(ctypes.byref(self.cfg), ctypes.byref(mt.s), _p(self.cells[e]),
                                    _p(self.visits[e]), _p(self.explored[e]), _p(self.scal[e]))
        if rc != 0:
            raise ValueError("Not enough available positions")

    def reset_philox(self, e, seed, env_id, episode):
        rc = lib().po_reset_philox(ctypes.byref(self.cfg), seed, env_id, episode, _p(self.cells[e]),
                                   _p(self.visits[e]), _p(self.explored[e]), _p(self.scal[e]))
        if rc != 0:
            raise ValueError("Not enough available positions")


def philox4x32(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().po_philox4x32(_p(c), _p(k), _p(o))
    return o


def pyset_free_list(G, obstacle_mask):
    m = np.ascontiguousarray(obstacle_mask, np.uint8).reshape(-1)
    out = np.zeros(G * G, np.int32)
    n = lib().po_pyset_free_list(G, _p(m), _p(out))
    return out[:n]


def synth_action(seed, env_id, t):
    return lib().po_synth_action(seed, env_id, t)


def bench(cfg, n_envs, steps, seed=0, threads=0):
    secs = ctypes.c_double(0.0)
    chk = lib().po_bench(ctypes.byref(cfg), n_envs, steps, seed, threads, ctypes.byref(secs))
    return secs.value, chk
