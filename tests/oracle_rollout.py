"""Oracle-side drivers used as the CHECKER by the GPU parity tests (test infra)."""
import numpy as np

from oracle import oracle as O


def scal_from_fixture(scal6, n):
    s = np.zeros((n, O.NSCAL), np.int32)
    s[:, :6] = scal6
    return s


class OracleVec:
    """Device-rng (Philox) DummyVecEnv-style rollout of selected global env ids,
    mirroring pe_create (all envs reset with episode 0) + pe_step(autoreset)."""

    def __init__(self, cfg_tuple, env_ids, seed, max_steps=1000):
        self.cfg = O.config(*cfg_tuple, max_steps=max_steps)
        self.ids = np.asarray(env_ids, np.int64)
        self.seed = seed
        self.b = O.Batch(self.cfg, len(self.ids))
        for k, e in enumerate(self.ids):
            self.b.reset_philox(k, seed, int(e), 0)
        self.ret = np.zeros(len(self.ids), np.float64)

    def obs(self):
        return self.b.obs()

    def step(self, actions):
        obs, rew, te, tr = self.b.step(actions)
        term_obs = obs.copy()
        done = te | tr
        self.ret += rew
        ep_ret = self.ret.copy()
        ep_len = self.b.scal[:, O.S_STEP].copy()
        for k in np.nonzero(done)[0]:
            self.b.reset_philox(int(k), self.seed, int(self.ids[k]), int(self.b.scal[k, O.S_EPISODE]))
            self.ret[k] = 0.0
        if done.any():
            fresh = self.b.obs(np.nonzero(done)[0])
            obs[done] = fresh[done]
        return obs, rew, te, tr, term_obs, ep_ret, ep_len
