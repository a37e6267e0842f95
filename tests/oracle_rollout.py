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

    def __init__(self, cfg_tuple, env_ids, seed, max_steps=1000, map_algo=0):
        self.cfg = O.config(*cfg_tuple, max_steps=max_steps, map_algo=map_algo)
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


class OracleBatch:
    """CPU stand-in with PlantOSBatch's interface, backed by the oracle (TEST INFRA:
    lets the host-side vec-env logic run and be checked without a GPU)."""

    def __init__(self, n, grid_size, num_plants, num_obstacles, lidar_range, lidar_channels, seed=0,
                 max_steps=1000, obs_codes=False):
        import torch
        self.torch = torch
        self.obs_codes = bool(obs_codes)  # io holds byte codes (plantos_amd/codes.py), as PlantOSBatch's
        self.device = torch.device("cpu")
        self.num_envs = n
        self.grid_size = grid_size
        self.cfg_t = (grid_size, num_plants, num_obstacles, lidar_range, lidar_channels)
        self.ov = OracleVec(self.cfg_t, np.arange(n), seed, max_steps=max_steps)
        self.obs_dim = O.obs_dim(self.ov.cfg)
        D = self.obs_dim
        self.obs = torch.as_tensor(self.ov.obs())
        self.reward = torch.zeros(n, dtype=torch.float32)
        self.terminated = torch.zeros(n, dtype=torch.uint8)
        self.truncated = torch.zeros(n, dtype=torch.uint8)
        self.terminal_obs = torch.zeros((n, D), dtype=torch.float32)
        self.episode_return = torch.zeros(n, dtype=torch.float64)
        self.episode_length = torch.zeros(n, dtype=torch.int32)
        self.terminal_info = torch.zeros((n, 11), dtype=torch.int32)
        self.seed_value = seed

    def _info_rows(self):
        b = self.ov.b
        rows = np.zeros((self.num_envs, 11), np.int32)
        for e in range(self.num_envs):
            th, hy, tot, ex, tc = b.info(e)
            s = b.scal[e]
            rows[e] = [s[O.S_X], s[O.S_Y], th, hy, tot, s[O.S_STEP], ex, tc, s[O.S_COLLIDED], s[O.S_COLL],
                       s[O.S_POISONED]]
        return rows

    def reset(self, mask=None):
        for e in range(self.num_envs):
            if mask is None or mask[e]:
                self.ov.b.reset_philox(e, self.ov.seed, int(self.ov.ids[e]), int(self.ov.b.scal[e, O.S_EPISODE]))
                self.ov.ret[e] = 0.0
        self.obs = self.torch.as_tensor(self.ov.obs())
        return self.obs

    # PlantOSBatch's packed output buffer: obs f32 [n, D] (or codes u8 [n, D]) | reward f32 |
    # term u8 | trunc u8
    def _io_offsets(self):
        n, D = self.num_envs, self.obs_dim
        if self.obs_codes:
            from plantos_amd.codes import io_layout
            return io_layout(n, D)
        return 4 * n * D, 4 * n * (D + 1), 4 * n * (D + 1) + n, 4 * n * (D + 1) + 2 * n

    def io_bytes(self):
        return self._io_offsets()[3]

    def new_io(self):
        return self.torch.zeros(self.io_bytes(), dtype=self.torch.uint8)

    def io_views(self, io):
        n, D = self.num_envs, self.obs_dim
        ro, to, tro, _ = self._io_offsets()
        obs = io[:n * D].view(n, D) if self.obs_codes else io[:ro].view(self.torch.float32).view(n, D)
        return obs, io[ro:to].view(self.torch.float32), io[to:tro], io[tro:tro + n]

    def _io_values(self, outs):
        """the step's outputs as the io holds them (obs encoded in code mode)"""
        if not self.obs_codes:
            return outs
        from plantos_amd.codes import encode_obs
        G, _, _, R, C = self.cfg_t
        return (self.torch.as_tensor(encode_obs(outs[0].numpy(), G, C, R)),) + tuple(outs[1:])

    @property
    def io(self):
        io = self.new_io()
        for dst, src in zip(self.io_views(io), self._io_values((self.obs, self.reward, self.terminated,
                                                                self.truncated))):
            dst.copy_(src)
        return io

    def expand_codes(self, src, blocks=1, obs=None, reward=None, terminated=None, truncated=None):
        """host twin of PlantOSBatch.expand_codes (plantos_amd/codes.py expand_host)"""
        from plantos_amd.codes import code_table, expand_host
        G, _, _, R, _ = self.cfg_t
        n, D = self.num_envs, self.obs_dim
        if obs is None:
            obs = self.torch.empty((blocks * n, D), dtype=self.torch.float32)
        expand_host(src.numpy(), blocks, n, D, self.io_bytes(), code_table(G, R), obs.numpy(),
                    None if reward is None else reward.numpy(), None if terminated is None else terminated.numpy(),
                    None if truncated is None else truncated.numpy())
        return obs, reward, terminated, truncated

    def step(self, actions, io=None):
        if io is not None:
            outs = self.step(actions)
            for dst, src in zip(self.io_views(io), self._io_values(outs)):
                dst.copy_(src)
            return self.io_views(io)
        a = np.asarray(actions.cpu().numpy() if hasattr(actions, "cpu") else actions, np.int64)
        pre_info = None
        obs, rew, te, tr, tobs, ret, ln = None, None, None, None, None, None, None
        # terminal info = info of the post-step, pre-reset state: step without reset first
        b = self.ov.b
        o, r, t1, t2 = b.step(a)
        pre_info = self._info_rows()
        done = t1 | t2
        self.ov.ret += r
        ret = self.ov.ret.copy()
        ln = b.scal[:, O.S_STEP].copy()
        tobs = o.copy()
        for k in np.nonzero(done)[0]:
            b.reset_philox(int(k), self.ov.seed, int(self.ov.ids[k]), int(b.scal[k, O.S_EPISODE]))
            self.ov.ret[k] = 0.0
        if done.any():
            o[done] = b.obs(np.nonzero(done)[0])[done]
        T = self.torch
        self.obs = T.as_tensor(o)
        self.reward = T.as_tensor(r.astype(np.float32))
        self.terminated = T.as_tensor(t1.astype(np.uint8))
        self.truncated = T.as_tensor(t2.astype(np.uint8))
        self.terminal_obs[done] = T.as_tensor(tobs[done])
        self.episode_return[done] = T.as_tensor(ret[done])
        self.episode_length[done] = T.as_tensor(ln[done].astype(np.int32))
        self.terminal_info[done] = T.as_tensor(pre_info[done])
        return self.obs, self.reward, self.terminated, self.truncated

    def get_info(self):
        return self.torch.as_tensor(self._info_rows())

    def get_state(self, parts=None):
        b = self.ov.b
        T = self.torch
        return {"cells": T.as_tensor(b.cells.copy()), "visits": T.as_tensor(b.visits.copy()),
                "explored": T.as_tensor(b.explored.copy()), "scalars": T.as_tensor(b.scal.copy())}

    def set_state(self, cells=None, visits=None, explored=None, scalars=None):
        b = self.ov.b
        if cells is not None:
            b.cells[...] = np.asarray(cells)
        if visits is not None:
            b.visits[...] = np.asarray(visits)
        if explored is not None:
            b.explored[...] = np.asarray(explored)
        if scalars is not None:
            b.scal[...] = np.asarray(scalars)

    def seed(self, seed, reset_episode_counters=True):
        self.ov.seed = seed
        if reset_episode_counters:
            self.ov.b.scal[:, O.S_EPISODE] = 0

    def close(self):
        pass
