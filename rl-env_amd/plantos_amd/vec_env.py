"""Drop-in vectorized-env faces over PlantOSBatch.

PlantOSVecEnv    -- the Stable-Baselines3 ``VecEnv`` protocol, replacing
                    ``DummyVecEnv([Monitor(PlantOSEnv(**kw)) ...])`` at
                    A2C_training.py:216-218 (also trainingCode.py:130,216).
                    Subclasses ``stable_baselines3.common.vec_env.VecEnv`` when SB3
                    is importable; otherwise it duck-types the same surface.
PlantOSVectorEnv -- the gymnasium-0.29 ``VectorEnv`` step/reset convention
                    (``final_observation`` / ``final_info`` on auto-reset).

Semantics mirrored:
  * ``step_wait`` auto-resets done envs (``done = terminated or truncated``); the
    returned obs row of a done env is its post-reset obs, the pre-reset obs is in
    ``infos[i]["terminal_observation"]`` and ``infos[i]["TimeLimit.truncated"] =
    truncated and not terminated`` (SB3 DummyVecEnv.step_wait).
  * ``infos[i]`` is PlantOSEnv._get_info() (plantos_env.py:317-336) of the step's
    final state -- for a done env, of the state BEFORE the reset -- plus, on done,
    Monitor's ``"episode": {"r", "l", "t"}`` (A2C_training.py:124 wraps each env in
    Monitor; r is the f64 sum of the step rewards, rounded to 6 decimals).
  * rewards are float32, dones bool, obs float32 [N, 5C+27].
  * ``seed(s)`` re-keys the device map generator (the reference ignores reset
    seeds for map layout, plantos_env.py:127 vs 344-372).

``infos`` is a lazy list: dicts are built on first access from one device->host
copy of the [N, 11] info table, so a training loop that never reads them pays
nothing.  With ``tensors=True`` obs/rewards/dones stay device tensors (zero-copy
hand-off to an on-GPU policy).
"""
import time

import numpy as np
import torch

from . import _capi as C
from .batch import PlantOSBatch

try:  # pragma: no cover - SB3 is not installed in this image
    from stable_baselines3.common.vec_env import VecEnv as _VecEnvBase
except Exception:  # noqa: BLE001
    _VecEnvBase = object

try:  # pragma: no cover - gymnasium is not installed in this image
    from gymnasium import spaces as _spaces
except Exception:  # noqa: BLE001
    _spaces = None


class Discrete:
    """Stand-in for gymnasium.spaces.Discrete (plantos_env.py:41) when gymnasium is absent."""

    def __init__(self, n, seed=None):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return int(self._rng.integers(self.n))

    def contains(self, x):
        return 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class Box:
    """Stand-in for gymnasium.spaces.Box (plantos_env.py:59-63) when gymnasium is absent."""

    def __init__(self, low, high, shape, dtype=np.float32, seed=None):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, self.dtype)
        self.high = np.full(self.shape, high, self.dtype)
        self._rng = np.random.default_rng(seed)

    def sample(self):
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box(0.0, 1.0, {self.shape}, {self.dtype})"


def make_spaces(obs_dim):
    if _spaces is not None:  # pragma: no cover
        return (_spaces.Box(low=0, high=1.0, shape=(obs_dim,), dtype=np.float32), _spaces.Discrete(5))
    return Box(0.0, 1.0, (obs_dim,), np.float32), Discrete(5)


def info_dict(row, lidar_range, lidar_channels):
    """PlantOSEnv._get_info() (plantos_env.py:317-336) from one pe_info row."""
    explored, total = int(row[C.PE_I_EXPLORED]), int(row[C.PE_I_TOTAL_CELLS])
    return {
        "rover_position": (int(row[C.PE_I_X]), int(row[C.PE_I_Y])),
        "thirsty_plants": int(row[C.PE_I_THIRSTY]),
        "hydrated_plants": int(row[C.PE_I_HYDRATED]),
        "total_plants": int(row[C.PE_I_TOTAL_PLANTS]),
        "step_count": int(row[C.PE_I_STEP]),
        "explored_cells": explored,
        "total_cells": total,
        "exploration_percentage": (np.float64(explored) / np.float64(total)) * 100 if total else float("nan"),
        "lidar_range": lidar_range,
        "lidar_channels": lidar_channels,
        "collided_with_wall": bool(row[C.PE_I_COLLIDED]),
        "total_collisions": int(row[C.PE_I_COLLISIONS]),
    }


class LazyInfos(list):
    """list of N info dicts, materialized per index on first access."""

    def __init__(self, n, build):
        super().__init__([None] * n)
        self._build = build

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        v = super().__getitem__(i)
        if v is None:
            v = self._build(i if i >= 0 else len(self) + i)
            super().__setitem__(i, v)
        return v

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]

    def get_table(self):
        return self._build.table()


class _StepView:
    """Host views of one step's device outputs, copied lazily (once each).

    The done/terminated/truncated flags are either host arrays already or a
    device u8 [2n] (terminated | truncated) copy fetched on first access (the
    zero-copy face: a loop that never reads infos never synchronizes)."""

    def __init__(self, venv, done_np=None, term_np=None, trunc_np=None, dev_flags=None):
        self.v = venv
        self._flags = None if dev_flags is not None else (done_np, term_np, trunc_np)
        self._dev_flags = dev_flags
        self._info = None
        self._tinfo = None
        self._tobs = None
        self._ret = None
        self._len = None
        self._didx = None
        self._t = round(time.time() - venv._t_start, 6)
        self._expired = False

    def _host_flags(self):
        if self._flags is None:
            f = self._dev_flags.cpu().numpy().astype(bool)  # own copy: valid after expiry
            n = f.shape[0] // 2
            te, tr = f[:n], f[n:]
            self._flags = (te | tr, te, tr)
        return self._flags

    @property
    def done(self):
        return self._host_flags()[0]

    @property
    def term(self):
        return self._host_flags()[1]

    @property
    def trunc(self):
        return self._host_flags()[2]

    @property
    def _done_idx(self):
        if self._didx is None:
            self._didx = np.nonzero(self.done)[0]
        return self._didx

    def expire(self):
        """The next step overwrites the device buffers this view reads lazily."""
        self._expired = True

    def _check(self):
        if self._expired:
            raise RuntimeError("infos of a previous step must be read before the next step() "
                               "(they are built lazily from device buffers)")

    def table(self):
        if self._info is None:
            self._check()
            self._info = self.v.batch.get_info().cpu().numpy()
        return self._info

    def _terminal(self):
        if self._tinfo is None:
            self._check()
            b = self.v.batch
            idx = torch.as_tensor(self._done_idx, device=b.device)
            self._tinfo = b.terminal_info.index_select(0, idx).cpu().numpy()
            self._tobs = b.terminal_obs.index_select(0, idx).cpu().numpy()
            self._ret = b.episode_return.index_select(0, idx).cpu().numpy()
            self._len = b.episode_length.index_select(0, idx).cpu().numpy()
        return self._tinfo, self._tobs, self._ret, self._len

    def __call__(self, i):
        R, Cc = self.v.lidar_range, self.v.lidar_channels
        if not self.done[i]:
            return info_dict(self.table()[i], R, Cc)
        k = int(np.searchsorted(self._done_idx, i))
        tinfo, tobs, ret, ln = self._terminal()
        d = info_dict(tinfo[k], R, Cc)
        d["terminal_observation"] = tobs[k]
        d["TimeLimit.truncated"] = bool(self.trunc[i] and not self.term[i])
        d["episode"] = {"r": round(float(ret[k]), 6), "l": int(ln[k]), "t": self._t}
        return d


class PlantOSVecEnv(_VecEnvBase):
    """SB3 VecEnv over N PlantOS envs resident in HBM (drop-in for DummyVecEnv).

    Constructor arguments mirror PlantOSEnv.__init__ (plantos_env.py:25-27) plus
    the batch size; env_kwargs from A2C_training.py:206-212 pass straight through:
        PlantOSVecEnv(512, **env_kwargs)
    """

    def __init__(self, num_envs, grid_size=21, num_plants=8, num_obstacles=50, lidar_range=2, lidar_channels=10,
                 thirsty_plant_prob=0.7, max_steps=1000, seed=0, device=None, tensors=False, env_id_offset=0,
                 observation_mode="lidar", render_mode=None, batch=None, reset_mode="device", python_seed=None,
                 curriculum=False, map_generation_algo="original", host_buffers=0, prefetch_every=None):
        """reset_mode="device": maps from the device generator keyed by (seed, env id,
        episode) -- the throughput mode.  reset_mode="cpython": the reference's own
        layouts, seed-exact: CPython's global `random` after random.seed(python_seed)
        (default: seed), consumed in DummyVecEnv order (pe_pystream, host side).
        curriculum=True (or "a2c") applies the batched CurriculumWrapper of
        A2C_training.py:37-109 to every env, as make_env_wrapper(use_curriculum=True)
        does (A2C_training.py:114-126); curriculum="trainingCode" the variant of
        trainingCode.py:24-98 (threshold marks the maze completed without
        terminating; 30 / 100 / +5, 50 episodes per maze) as its make_env_wrapper
        does (trainingCode.py:103-111); a dict {"variant": ..., **CurriculumWrapper
        arguments} overrides the defaults.
        map_generation_algo="maze" selects the fork's maze layouts
        (gradio-app/plantos_env_new.py:28, 408-604) in either reset mode.
        host_buffers=k (numpy face): obs arrive in a ring of k pinned host buffers
        (one DMA at full PCIe rate; each returned obs array stays valid for k steps,
        enough for SB3's collect_rollouts with k >= 2); 0 (default): a fresh array
        per step, as DummyVecEnv returns.
        prefetch_every: pe_config.prefetch_every (steps between the launches that
        generate next-episode maps ahead of time; None: the library's 256, 0: off)."""
        if observation_mode != "lidar":
            raise ValueError("only observation_mode='lidar' exists in the reference (plantos_env.py:27)")
        if reset_mode not in ("device", "cpython"):
            raise ValueError("reset_mode must be 'device' or 'cpython'")
        self.reset_mode = reset_mode
        self.batch = batch if batch is not None else PlantOSBatch(
            num_envs, grid_size=grid_size, num_plants=num_plants, num_obstacles=num_obstacles,
            lidar_range=lidar_range, lidar_channels=lidar_channels, thirsty_plant_prob=thirsty_plant_prob,
            max_steps=max_steps, autoreset=reset_mode == "device", seed=seed, env_id_offset=env_id_offset,
            device=device, map_generation_algo=map_generation_algo, prefetch_every=prefetch_every)
        if curriculum:
            # True / "a2c": A2C_training.py:37-109 as :121 builds it; "trainingCode":
            # trainingCode.py:24-98 as :107 builds it; a dict: {"variant": ..., overrides}
            kw = dict(curriculum) if isinstance(curriculum, dict) else {}
            variant = curriculum if isinstance(curriculum, str) else kw.pop("variant", "a2c")
            self.batch.enable_curriculum(variant, **kw)
        self.curriculum = bool(curriculum)
        self._pystream = None
        if reset_mode == "cpython":
            self._pystream = C.PyStream(grid_size, num_plants, num_obstacles,
                                        seed if python_seed is None else python_seed, thirsty_plant_prob,
                                        getattr(self.batch, "map_generation_algo", "original"))
        self.grid_size, self.num_plants, self.num_obstacles = grid_size, num_plants, num_obstacles
        self.lidar_range, self.lidar_channels = lidar_range, lidar_channels
        self.thirsty_plant_prob, self.max_steps = thirsty_plant_prob, max_steps
        self.render_mode = render_mode
        self.tensors = bool(tensors)
        self.host_buffers = int(host_buffers)
        self._pinned_packed = None
        self._pinned_obs = None
        self._ring = 0
        obs_space, act_space = make_spaces(self.batch.obs_dim)
        if _VecEnvBase is not object:  # pragma: no cover
            super().__init__(num_envs, obs_space, act_space)
        self.num_envs = int(num_envs)
        self.observation_space, self.action_space = obs_space, act_space
        self.reset_infos = [{} for _ in range(self.num_envs)]
        self._last_view = None
        self._actions = None
        self._t_start = time.time()
        self._seed = seed

    # ------------------------------------------------------------------ helpers
    def _out(self, t):
        return t if self.tensors else t.cpu().numpy()

    # ------------------------------------------------------------------ VecEnv API
    def _load_stream_maps(self, idx):
        """Next len(idx) CPython-stream maps into envs idx (ascending), obs rows updated."""
        cells, rover = self._pystream.next(len(idx))
        fresh = self.batch.load_maps(idx, cells, rover)
        self.batch.obs[torch.as_tensor(idx, device=self.batch.device)] = fresh

    def _new_view(self, done_np=None, te_np=None, tr_np=None, dev_flags=None):
        if self._last_view is not None:
            self._last_view.expire()
        self._last_view = _StepView(self, done_np, te_np, tr_np, dev_flags=dev_flags)
        return self._last_view

    def _to_host(self, obs):
        """(obs, reward, terminated, truncated) as numpy with ONE stream sync: the
        packed per-step scalars go to a pinned buffer asynchronously, the obs
        either into the pinned ring (host_buffers > 0: views valid for that many
        steps) or into a fresh array (obs.cpu(), which synchronizes the stream
        after both copies)."""
        b = self.batch
        packed = getattr(b, "packed_outputs", None)
        if packed is None or not packed.is_cuda:  # e.g. the oracle-backed batch of the CPU tests
            return (obs.cpu().numpy(), b.reward.cpu().numpy(), b.terminated.cpu().numpy().astype(bool),
                    b.truncated.cpu().numpy().astype(bool))
        n = self.num_envs
        if self._pinned_packed is None:
            self._pinned_packed = torch.empty(packed.shape, dtype=torch.uint8, pin_memory=True)
        hp = self._pinned_packed
        hp.copy_(packed, non_blocking=True)
        if self.host_buffers:
            if self._pinned_obs is None:
                self._pinned_obs = [torch.empty(obs.shape, dtype=obs.dtype, pin_memory=True)
                                    for _ in range(self.host_buffers)]
            ho = self._pinned_obs[self._ring]
            self._ring = (self._ring + 1) % self.host_buffers
            ho.copy_(obs, non_blocking=True)
            torch.cuda.current_stream(b.device).synchronize()
            obs_np = ho.numpy()
        else:
            obs_np = obs.cpu().numpy()
        hn = hp.numpy()
        rew = hn[:4 * n].view(np.float32).copy()
        te = hn[4 * n:5 * n].astype(bool)
        tr = hn[5 * n:].astype(bool)
        return obs_np, rew, te, tr

    def reset(self):
        """All envs get a fresh map; returns obs [N, D]."""
        if self._last_view is not None:
            self._last_view.expire()
        if self.reset_mode == "cpython":
            self._load_stream_maps(np.arange(self.num_envs))
            obs = self.batch.obs
        else:
            obs = self.batch.reset()
        z = np.zeros(self.num_envs, bool)
        self.reset_infos = LazyInfos(self.num_envs, self._new_view(z, z, z))
        return self._out(obs.clone() if self.tensors else obs)

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        a = self._actions
        if self._last_view is not None:
            self._last_view.expire()
        if isinstance(a, np.ndarray) or not isinstance(a, torch.Tensor):
            a = torch.as_tensor(np.asarray(a).reshape(-1).astype(np.int64), device=self.batch.device)
        obs, rew, te, tr = self.batch.step(a.reshape(-1))
        self._actions = None
        if self.reset_mode == "cpython":  # DummyVecEnv: done envs reset in index order
            idx = torch.nonzero(te.bool() | tr.bool()).reshape(-1).cpu().numpy()
            if len(idx):
                self._load_stream_maps(idx)
        if self.tensors:
            n = self.num_envs
            packed = getattr(self.batch, "packed_outputs", None)
            flags = packed[4 * n:].clone() if packed is not None else torch.cat([te, tr]).to(torch.uint8)
            infos = LazyInfos(n, self._new_view(dev_flags=flags))
            return obs.clone(), rew.clone(), (te | tr).bool(), infos
        obs_np, rew_np, te_np, tr_np = self._to_host(obs)
        done_np = te_np | tr_np
        infos = LazyInfos(self.num_envs, self._new_view(done_np, te_np, tr_np))
        return obs_np, rew_np, done_np, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.batch.close()
        if self._pystream is not None:
            self._pystream.close()

    def seed(self, seed=None):
        """Re-key the device map generator; per-env seeds seed+i like DummyVecEnv."""
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 31 - 1))
        self._seed = int(seed)
        self.batch.seed(int(seed))
        if self.reset_mode == "cpython":  # random.seed(seed) of the reference's global stream
            self._pystream.close()
            self._pystream = C.PyStream(self.grid_size, self.num_plants, self.num_obstacles, int(seed),
                                        self.thirsty_plant_prob,
                                        getattr(self.batch, "map_generation_algo", "original"))
        return [int(seed) + i for i in range(self.num_envs)]

    def _indices(self, indices):
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    # attributes of PlantOSEnv a caller may read (MCTS clone set mcts_custom_trainer.py:236-241,
    # CurriculumWrapper visit_counts A2C_training.py:88-93)
    def get_attr(self, attr_name, indices=None):
        idx = self._indices(indices)
        const = {"grid_size": self.grid_size, "num_plants": self.num_plants, "num_obstacles": self.num_obstacles,
                 "lidar_range": self.lidar_range, "lidar_channels": self.lidar_channels,
                 "thirsty_plant_prob": self.thirsty_plant_prob, "max_steps": self.max_steps,
                 "observation_space": self.observation_space, "action_space": self.action_space,
                 "render_mode": self.render_mode}
        if attr_name in const:
            return [const[attr_name] for _ in idx]
        st = self.batch.get_state()
        cells = st["cells"].cpu().numpy()
        sc = st["scalars"].cpu().numpy()
        if attr_name in ("exploration_threshold", "episode_count", "successful_explorations",
                         "episodes_on_current_maze", "maze_completed") and self.curriculum:
            thr, cnt = self.batch.get_curriculum()
            thr, cnt = thr.cpu().numpy(), cnt.cpu().numpy()
            col = {"episode_count": 0, "successful_explorations": 1, "episodes_on_current_maze": 2}
            if attr_name == "exploration_threshold":
                return [float(thr[i]) for i in idx]
            if attr_name == "maze_completed":
                return [bool(cnt[i, 3] & 1) for i in idx]
            return [int(cnt[i, col[attr_name]]) for i in idx]
        if attr_name == "visit_counts":
            v = st["visits"].cpu().numpy()
            return [v[i].copy() for i in idx]
        if attr_name == "explored_map":
            x = st["explored"].cpu().numpy()
            return [x[i].copy() for i in idx]
        if attr_name == "rover_pos":
            return [(int(sc[i, C.PE_S_X]), int(sc[i, C.PE_S_Y])) for i in idx]
        if attr_name == "step_count":
            return [int(sc[i, C.PE_S_STEP]) for i in idx]
        if attr_name == "total_collisions":
            return [int(sc[i, C.PE_S_COLL]) for i in idx]
        if attr_name == "collided_with_wall":
            return [bool(sc[i, C.PE_S_COLLIDED]) for i in idx]
        if attr_name == "completion_bonus_given":
            return [bool(sc[i, C.PE_S_BONUS]) for i in idx]
        if attr_name == "obstacles":
            return [{(int(r), int(c)) for r, c in zip(*np.nonzero(cells[i] == C.PE_CELL_OBSTACLE))} for i in idx]
        if attr_name == "plants":
            out = []
            for i in idx:
                d = {}
                for r, c in zip(*np.nonzero(cells[i] >= C.PE_CELL_HYDRATED)):
                    d[(int(r), int(c))] = bool(cells[i][r, c] == C.PE_CELL_THIRSTY)
                out.append(d)
            return out
        raise AttributeError(f"PlantOSVecEnv has no per-env attribute {attr_name!r}")

    def set_attr(self, attr_name, value, indices=None):
        idx = self._indices(indices)
        if attr_name != "visit_counts":
            raise AttributeError(f"set_attr supports 'visit_counts' only, not {attr_name!r}")
        st = self.batch.get_state()
        v = st["visits"].cpu().numpy()
        vals = value if isinstance(value, (list, tuple)) else [value] * len(idx)
        for i, val in zip(idx, vals):
            v[i] = np.asarray(val, np.int32)
        self.batch.set_state(visits=v)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        if method_name == "get_wrapper_attr":
            return self.get_attr(method_args[0], indices)
        raise AttributeError(f"env_method({method_name!r}) is not available on the batched env")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_images(self):
        raise NotImplementedError("rendering is out of scope (SURVEY.md §2 row 2)")

    def render(self, mode=None):
        raise NotImplementedError("rendering is out of scope (SURVEY.md §2 row 2)")


class PlantOSVectorEnv:
    """gymnasium-0.29 VectorEnv convention over the same batch:
    reset(seed) -> (obs, infos); step(a) -> (obs, rewards, terminations, truncations, infos),
    infos a dict of arrays with "final_observation" / "final_info" for done envs."""

    def __init__(self, num_envs, **kw):
        self.venv = PlantOSVecEnv(num_envs, **kw)
        self.num_envs = self.venv.num_envs
        self.single_observation_space = self.venv.observation_space
        self.single_action_space = self.venv.action_space

    def reset(self, seed=None, options=None):
        if seed is not None:
            self.venv.seed(seed)
        obs = self.venv.reset()
        return obs, {}

    def step(self, actions):
        obs, rew, done, infos = self.venv.step(actions)
        view = infos._build
        out_info = {}
        if done.any():
            final_obs = np.empty(self.num_envs, dtype=object)
            final_info = np.empty(self.num_envs, dtype=object)
            for i in np.nonzero(done)[0]:
                d = dict(infos[i])
                final_obs[i] = d.pop("terminal_observation")
                d.pop("TimeLimit.truncated", None)
                final_info[i] = d
            out_info = {"final_observation": final_obs, "_final_observation": np.asarray(done, bool),
                        "final_info": final_info, "_final_info": np.asarray(done, bool)}
        return obs, rew, view.term.copy(), view.trunc.copy(), out_info

    def close(self):
        self.venv.close()
