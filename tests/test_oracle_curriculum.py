"""The CurriculumWrapper restatement (test infrastructure, over the oracle) against
the reference's own wrappers: tests/golden/curriculum_*.npz were produced by the
reference class A2C_training.py:37-109, curriculum_tc_*.npz by trainingCode.py:24-98
(threshold marks the maze completed but does not terminate), around the reference
env (tools/gen_golden.py) in a DummyVecEnv loop.  Pins the semantics the device implements: threshold
termination, threshold increments, visit counts carried into the next episode
with the explored map restarted, and the stale reset obs."""
import numpy as np
import pytest

from golden_util import cfg_tuple, load
from oracle import oracle as O


class OracleCurriculumVec:
    """DummyVecEnv([CurriculumWrapper(env)]) over the oracle, CPython reset stream."""

    # constructor defaults of the two reference classes as their make_env_wrapper builds them
    VARIANTS = {"a2c": dict(initial=40.0, maximum=100.0, inc=10.0, max_eps=3, terminate=True),  # A2C_training.py:41-54
                "tc": dict(initial=30.0, maximum=100.0, inc=5.0, max_eps=50, terminate=False)}  # trainingCode.py:29-42

    def __init__(self, cfg, n, seed, initial=40.0, maximum=100.0, inc=10.0, max_eps=3, terminate=True):
        self.c = O.config(*cfg)
        self.b = O.Batch(self.c, n)
        self.mt = O.MT(seed)
        self.n = n
        self.thr = np.full(n, initial)
        self.maximum, self.inc, self.max_eps = maximum, inc, max_eps
        self.terminate = terminate
        self.episodes = np.zeros(n, np.int64)
        self.successes = np.zeros(n, np.int64)
        self.on_maze = np.zeros(n, np.int64)
        self.completed = np.zeros(n, bool)
        self.persistent = [None] * n

    def _new_map(self, e):
        """plantos_env.py:125-158 on the shared CPython stream (DummyVecEnv order)."""
        self.b.reset_cpython(e, self.mt)

    def reset_env(self, e):
        self.episodes[e] += 1
        self.on_maze[e] += 1
        timeout = self.on_maze[e] >= self.max_eps
        if self.completed[e] or timeout:
            if self.completed[e]:
                self.thr[e] = min(self.thr[e] + self.inc, self.maximum)
                self.successes[e] += 1
            self.completed[e] = False
            self.on_maze[e] = 0
            self._new_map(e)
            obs = self.b.obs([e])[e]
            self.persistent[e] = None
        else:
            self._new_map(e)
            obs = self.b.obs([e])[e]  # computed before the injection below
            if self.persistent[e] is not None:
                self.b.visits[e] = self.persistent[e].copy()
            else:
                self.persistent[e] = self.b.visits[e].copy()
        return obs

    def reset(self):
        return np.array([self.reset_env(e) for e in range(self.n)])

    def step(self, actions):
        obs, rew, te, tr = self.b.step(np.asarray(actions, np.int64))
        te = te.copy()
        tobs = obs.copy()
        ex = (self.b.explored > 0).reshape(self.n, -1).sum(1).astype(np.float64)        # plantos_env.py:320
        tc = (self.b.cells != 1).reshape(self.n, -1).sum(1).astype(np.float64)           # :321
        hit = (ex / tc) * 100 >= self.thr                                  # A2C_training.py:101, trainingCode.py:87
        self.completed |= hit
        if self.terminate:                                                  # A2C_training.py:103 only
            te |= hit
        for e in range(self.n):
            if self.persistent[e] is not None:
                self.persistent[e] = self.b.visits[e].copy()
        for e in range(self.n):
            if te[e] or tr[e]:
                obs[e] = self.reset_env(e)
        return obs, rew, te, tr, tobs


@pytest.mark.parametrize("name", ["curriculum_g20_explore", "curriculum_g7_explore", "curriculum_g20_random",
                                  "curriculum_tc_g20_explore", "curriculum_tc_g7_explore", "curriculum_tc_g20_random"])
def test_curriculum_restatement_matches_reference(name):
    """curriculum_*: A2C_training.py's wrapper; curriculum_tc_*: trainingCode.py's."""
    f = load(name)
    T, N = f["actions"].shape
    v = OracleCurriculumVec(cfg_tuple(f), N, int(f["seed"]),
                            **OracleCurriculumVec.VARIANTS["tc" if "_tc_" in name else "a2c"])
    assert (v.reset() == f["obs0"]).all()
    for t in range(T):
        obs, rew, te, tr, tobs = v.step(f["actions"][t])
        assert (rew == f["reward"][t]).all(), t
        assert (te == f["terminated"][t].astype(bool)).all() and (tr == f["truncated"][t].astype(bool)).all(), t
        done = te | tr
        assert (tobs[done] == f["terminal_obs"][t][done]).all(), t
        assert (obs == f["obs"][t]).all(), t
        assert (v.thr == f["threshold"][t]).all(), t
        assert (v.b.visits.reshape(N, -1).sum(1) == f["visits_sum"][t]).all(), t
    fin = np.stack([v.episodes, v.successes, v.on_maze,
                    v.completed.astype(int) | 2 * np.array([p is not None for p in v.persistent])], 1)
    assert (fin == f["final_counters"]).all()
    assert v.mt.u32() == int(f["next_u32"])
