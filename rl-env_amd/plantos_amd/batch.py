"""PlantOSBatch: N PlantOS envs resident in HBM, driven through the C-ABI.

torch is plumbing here: it owns the device buffers and supplies the HIP stream;
all env work runs in the HIP kernels of libplantos_hip.so.
"""
import ctypes

import torch

from . import _capi as C


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


class PlantOSBatch:
    """A batch of `num_envs` independent PlantOS envs on one GPU.

    Parameters mirror PlantOSEnv.__init__ (plantos_env.py:25-27) plus the batch
    size, device, the device-rng seed, and `env_id_offset` (global id of env 0,
    used when the batch is one shard of a multi-GPU job); `map_generation_algo`
    is the fork's ('original' or 'maze', gradio-app/plantos_env_new.py:28).
    `coop_max_done` / `prefetch_every` tune the auto-reset paths (pe_config; None =
    the library's choice); they change speed, never results.

    `obs_codes=True` (pe_config.obs_codes; geometries with a byte-coded sector
    kernel): the step writes the obs as byte codes (codes.py) -- the io buffer is
    codes u8 [n, D] | reward | terminated | truncated, `step()` returns the codes in
    place of the f32 obs, and `expand_codes` turns one or many such buffers (e.g.
    every rank's, gathered) into f32 in one kernel.  The host-boundary form of a
    sharded job (shard.py).
    """

    def __init__(self, num_envs, grid_size=21, num_plants=8, num_obstacles=50, lidar_range=2,
                 lidar_channels=10, thirsty_plant_prob=0.7, max_steps=1000, autoreset=True, seed=0,
                 env_id_offset=0, device=None, rewards=None, map_generation_algo="original",
                 coop_max_done=None, prefetch_every=None, obs_codes=False):
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device() if torch.cuda.is_available() else 0)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise C.PlantOSNativeError("PlantOSBatch needs a HIP device (no CPU fallback)")
        L = C.lib()
        cfg = C.default_config(grid_size, num_plants, num_obstacles, lidar_range, lidar_channels)
        cfg.thirsty_plant_prob = float(thirsty_plant_prob)
        cfg.max_steps = int(max_steps)
        cfg.autoreset = int(bool(autoreset))
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.env_id_offset = int(env_id_offset)
        cfg.map_generation_algo = C.map_algo_id(map_generation_algo)
        if coop_max_done is not None:
            cfg.coop_max_done = int(coop_max_done)
        if prefetch_every is not None:
            cfg.prefetch_every = int(prefetch_every)
        cfg.obs_codes = int(bool(obs_codes))
        self.obs_codes = bool(obs_codes)
        self.map_generation_algo = "maze" if cfg.map_generation_algo == C.PE_MAP_MAZE else "original"
        for k, v in (rewards or {}).items():
            setattr(cfg, k, float(v))
        self.cfg = cfg
        self.num_envs = int(num_envs)
        self.grid_size = grid_size
        self.obs_dim = int(L.pe_obs_dim(ctypes.byref(cfg)))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            C.check(L.pe_create(ctypes.byref(cfg), self.device.index or 0, self.num_envs, ctypes.byref(h)),
                    "pe_create")
        self._h = h
        n, D, dev = self.num_envs, self.obs_dim, self.device
        # one step's outputs in ONE device buffer (io): obs f32 [n, D] | reward f32 [n] |
        # terminated u8 [n] | truncated u8 [n].  A host-side consumer fetches the
        # per-step scalars with one copy, and a multi-GPU job gathers a whole step
        # with one collective (shard.py).
        self._io = self.new_io()
        self.obs, self.reward, self.terminated, self.truncated = self.io_views(self._io)
        self._packed = self._io[self._io_offsets()[0]:]
        self.terminal_obs = torch.zeros((n, D), dtype=torch.float32, device=dev)
        self.episode_return = torch.zeros(n, dtype=torch.float64, device=dev)
        self.episode_length = torch.zeros(n, dtype=torch.int32, device=dev)
        self.info_buf = torch.zeros((n, C.PE_NINFO), dtype=torch.int32, device=dev)
        self.terminal_info = torch.zeros((n, C.PE_NINFO), dtype=torch.int32, device=dev)
        self._dev_index = self.device.index or 0
        self._L = L
        self._out_ptrs = (self.reward.data_ptr(), self.terminated.data_ptr(), self.truncated.data_ptr())
        self._tobs_ptr = self.terminal_obs.data_ptr()
        self._ep_ptrs = (self.episode_return.data_ptr(), self.episode_length.data_ptr(),
                         self.terminal_info.data_ptr())
        self.raise_on_errors()

    def raise_on_errors(self):
        """Surface the reference's exceptions that the batch records per env:
        ValueError when a reset had no room (plantos_env.py:360-364)."""
        bits = self.poll_errors()
        if bits & 4:
            raise ValueError("Not enough available positions to place the plants and the rover "
                             "(plantos_env.py:360-364)")
        return bits

    # ----------------------------------------------------------------- plumbing
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @property
    def handle(self):
        if not self._h:
            raise ValueError("PlantOSBatch is closed")
        return self._h

    @property
    def io(self):
        """u8 device buffer of one step's outputs (see io_views)."""
        return self._io

    def _io_offsets(self):
        """(reward, terminated, truncated, total) byte offsets of the io buffer."""
        n, D = self.num_envs, self.obs_dim
        if self.obs_codes:
            from .codes import io_layout
            return io_layout(n, D)
        return 4 * n * D, 4 * n * (D + 1), 4 * n * (D + 1) + n, 4 * n * (D + 1) + 2 * n

    def io_bytes(self):
        return self._io_offsets()[3]

    def new_io(self):
        """A fresh output buffer for step(io=...) (e.g. double buffering)."""
        return torch.zeros(self.io_bytes(), dtype=torch.uint8, device=self.device)

    def io_views(self, io):
        """(obs f32 [n, D] -- or codes u8 [n, D] with obs_codes --, reward f32 [n],
        terminated u8 [n], truncated u8 [n]) views of io."""
        n, D = self.num_envs, self.obs_dim
        ro, to, tro, end = self._io_offsets()
        obs = io[:n * D].view(n, D) if self.obs_codes else io[:ro].view(torch.float32).view(n, D)
        return obs, io[ro:to].view(torch.float32), io[to:tro], io[tro:tro + n]

    def code_table(self):
        """float32[256] (host): the value of every obs byte code (pe_obs_code_table)."""
        import numpy as np
        t = np.zeros(256, np.float32)
        C.check(C.lib().pe_obs_code_table(self.handle, t.ctypes.data_as(ctypes.c_void_p)), "pe_obs_code_table")
        return t

    def expand_codes(self, src, blocks=1, obs=None, reward=None, terminated=None, truncated=None):
        """f32 obs (and, where given, reward / terminated / truncated) of `blocks` code-mode
        io buffers of this batch's size laid out back to back in `src` (a contiguous u8
        device tensor of blocks * io_bytes(), e.g. the root's gather buffer) -- one
        kernel, written straight into the given (or new) contiguous tensors."""
        n, D = self.num_envs, self.obs_dim
        stride = self.io_bytes()
        if not (type(src) is torch.Tensor and src.dtype is torch.uint8 and src.is_cuda and src.is_contiguous()
                and src.numel() == blocks * stride):
            raise ValueError(f"src must be a contiguous uint8 device tensor of {blocks} x {stride} bytes")
        if obs is None:
            obs = torch.empty((blocks * n, D), dtype=torch.float32, device=self.device)
        # the kernel writes blocks*n rows of D floats and blocks*n per-env values through raw
        # pointers: every output must be exactly that, on this batch's device
        rows = blocks * n
        for name, t, dt, shape in (("obs", obs, torch.float32, (rows, D)), ("reward", reward, torch.float32, (rows,)),
                                   ("terminated", terminated, torch.uint8, (rows,)),
                                   ("truncated", truncated, torch.uint8, (rows,))):
            if t is None:
                continue
            if not (type(t) is torch.Tensor and t.dtype is dt and t.is_cuda and t.get_device() == self._dev_index
                    and t.is_contiguous() and tuple(t.shape) == shape):
                raise ValueError(f"{name} must be a contiguous {dt} tensor of shape {shape} on {self.device}")
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_expand_obs_codes(self.handle, int(blocks), n, _ptr(src), stride, _ptr(obs), _ptr(reward),
                                                _ptr(terminated), _ptr(truncated), self._stream()),
                    "pe_expand_obs_codes")
        return obs, reward, terminated, truncated

    @property
    def packed_outputs(self):
        """u8 [6n] device view of one step's scalars: reward (f32 [n]) |
        terminated (u8 [n]) | truncated (u8 [n])."""
        return self._packed

    @property
    def kernel_name(self):
        return C.lib().pe_kernel_name(self.handle).decode()

    @property
    def prefetch_every(self):
        """Steps between the launches that generate next-episode maps ahead of time
        (0: no prefetched resets for this geometry / configuration)."""
        return int(C.lib().pe_prefetch_every(self.handle))

    @property
    def kernel_variant(self):
        return int(C.lib().pe_kernel_variant(self.handle))

    @property
    def state_bytes(self):
        return int(C.lib().pe_state_bytes(self.handle))

    def close(self):
        if getattr(self, "_h", None):
            C.check(C.lib().pe_destroy(self._h), "pe_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ----------------------------------------------------------------- hot path
    def reset(self, mask=None, obs=None):
        """Reset masked envs (all if mask is None); returns obs [n, D] (device, f32;
        with obs_codes a new f32 tensor unless `obs` is given)."""
        if obs is None and self.obs_codes:
            obs = torch.empty((self.num_envs, self.obs_dim), dtype=torch.float32, device=self.device)
        out = self.obs if obs is None else obs
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_reset(self.handle, _ptr(m), _ptr(out), self._stream()), "pe_reset")
        return out

    def step(self, actions, obs=None, want_terminal_obs=True, io=None):
        """One step of every env. `actions`: int32/int64 tensor [n] on the device
        (other inputs are converted).  Returns device tensors
        (obs, reward, terminated, truncated).  Asynchronous on torch's current
        stream (graph-capturable); the library binds and restores the device.
        io: another output buffer (new_io()) to write this step's outputs to."""
        if io is not None:
            if not (type(io) is torch.Tensor and io.dtype is torch.uint8 and io.is_cuda
                    and io.get_device() == self._dev_index and io.is_contiguous()
                    and io.numel() == self.io_bytes()):
                raise ValueError(f"io must be a contiguous uint8 tensor of {self.io_bytes()} bytes on {self.device} "
                                 "(PlantOSBatch.new_io())")
            o, r_, te_, tr_ = self.io_views(io)
            step = self._L.pe_step_codes if self.obs_codes else self._L.pe_step
            rc = step(self.handle, self._actions_ptr(actions), self._act_bytes, o.data_ptr(),
                                 r_.data_ptr(), te_.data_ptr(), tr_.data_ptr(),
                                 self._tobs_ptr if want_terminal_obs else None, self._ep_ptrs[0], self._ep_ptrs[1],
                                 self._ep_ptrs[2], torch.cuda.current_stream(self._dev_index).cuda_stream)
            if rc:
                C.check(rc, "pe_step_codes" if self.obs_codes else "pe_step")
            return o, r_, te_, tr_
        a = actions
        if not (type(a) is torch.Tensor and a.is_cuda and a.get_device() == self._dev_index
                and (a.dtype is torch.int32 or a.dtype is torch.int64) and a.is_contiguous()):
            a = torch.as_tensor(a).to(device=self.device, dtype=torch.int64).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.numel()}")
        out = self.obs if obs is None else obs
        if self.obs_codes and obs is not None:
            raise ValueError("obs_codes: the step writes codes into the io buffer (expand_codes for f32)")
        r, te, tr = self._out_ptrs
        step = self._L.pe_step_codes if self.obs_codes else self._L.pe_step
        rc = step(self.handle, a.data_ptr(), a.element_size(), out.data_ptr(), r, te, tr,
                             self._tobs_ptr if want_terminal_obs else None, self._ep_ptrs[0], self._ep_ptrs[1],
                             self._ep_ptrs[2], torch.cuda.current_stream(self._dev_index).cuda_stream)
        if rc:
            C.check(rc, "pe_step_codes" if self.obs_codes else "pe_step")
        return out, self.reward, self.terminated, self.truncated

    def _actions_ptr(self, actions):
        a = actions
        if not (type(a) is torch.Tensor and a.is_cuda and a.get_device() == self._dev_index
                and (a.dtype is torch.int32 or a.dtype is torch.int64) and a.is_contiguous()):
            a = torch.as_tensor(a).to(device=self.device, dtype=torch.int64).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.numel()}")
        self._a_keep = a  # alive until the launch has read it
        self._act_bytes = a.element_size()
        return a.data_ptr()

    # ----------------------------------------------------------------- inspection
    def get_info(self):
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_get_info(self.handle, _ptr(self.info_buf), self._stream()), "pe_get_info")
        return self.info_buf

    def get_state(self, parts=("cells", "visits", "explored", "scalars")):
        """Canonical state in the reference's terms (plantos_env.py:96-123); `parts`
        selects which arrays to export (the rest are not materialized)."""
        n, G = self.num_envs, self.grid_size
        dev = self.device
        cells = torch.empty((n, G, G), dtype=torch.uint8, device=dev) if "cells" in parts else None
        visits = torch.empty((n, G, G), dtype=torch.int32, device=dev) if "visits" in parts else None
        explored = torch.empty((n, G, G), dtype=torch.int8, device=dev) if "explored" in parts else None
        scal = torch.empty((n, C.PE_NSCAL), dtype=torch.int32, device=dev) if "scalars" in parts else None
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_get_state(self.handle, _ptr(cells), _ptr(visits), _ptr(explored), _ptr(scal),
                                         self._stream()), "pe_get_state")
        out = {"cells": cells, "visits": visits, "explored": explored, "scalars": scal}
        return {k: v for k, v in out.items() if v is not None}

    def set_state(self, cells=None, visits=None, explored=None, scalars=None):
        def dev(x, dt):
            return None if x is None else torch.as_tensor(x).to(device=self.device, dtype=dt).contiguous()
        c, v, e, s = dev(cells, torch.uint8), dev(visits, torch.int32), dev(explored, torch.int8), dev(
            scalars, torch.int32)
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_set_state(self.handle, _ptr(c), _ptr(v), _ptr(e), _ptr(s), self._stream()),
                    "pe_set_state")
        torch.cuda.current_stream(self.device).synchronize()

    def load_maps(self, env_index, cells, rover):
        """Reset envs `env_index` to given layouts; returns their obs [k, D]."""
        idx = torch.as_tensor(env_index).to(device=self.device, dtype=torch.int32).contiguous()
        cl = torch.as_tensor(cells).to(device=self.device, dtype=torch.uint8).contiguous()
        rv = torch.as_tensor(rover).to(device=self.device, dtype=torch.int32).contiguous()
        k = idx.numel()
        out = torch.empty((k, self.obs_dim), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_load_maps(self.handle, k, _ptr(idx), _ptr(cl), _ptr(rv), _ptr(out), self._stream()),
                    "pe_load_maps")
        return out

    def synth_actions(self, seed, t, out=None):
        out = torch.empty(self.num_envs, dtype=torch.int32, device=self.device) if out is None else out
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_synth_actions(self.handle, int(seed), int(t), _ptr(out), self._stream()),
                    "pe_synth_actions")
        return out

    def poll_errors(self):
        bits = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_poll_errors(self.handle, ctypes.byref(bits), self._stream()), "pe_poll_errors")
        return int(bits.value)

    # ----------------------------------------------------------------- curriculum
    # the reference's two CurriculumWrapper classes: constructor defaults as their
    # make_env_wrapper builds them (A2C_training.py:41-54,121; trainingCode.py:29-42,107)
    CURRICULUM_VARIANTS = {
        "a2c": dict(initial_threshold=40.0, max_threshold=100.0, threshold_increment=10.0,
                    max_episodes_per_maze=3, terminate_on_threshold=True),
        "trainingCode": dict(initial_threshold=30.0, max_threshold=100.0, threshold_increment=5.0,
                             max_episodes_per_maze=50, terminate_on_threshold=False),
    }

    def enable_curriculum(self, variant="a2c", **overrides):
        """Batched CurriculumWrapper on every env.  variant="a2c": A2C_training.py:37-109
        (reaching the threshold terminates the episode); variant="trainingCode":
        trainingCode.py:24-98 (it only marks the maze completed).  Keyword overrides:
        initial_threshold, max_threshold, threshold_increment, max_episodes_per_maze,
        terminate_on_threshold."""
        if variant not in self.CURRICULUM_VARIANTS:
            raise ValueError(f"curriculum variant must be one of {sorted(self.CURRICULUM_VARIANTS)}")
        kw = dict(self.CURRICULUM_VARIANTS[variant])
        unknown = set(overrides) - set(kw)
        if unknown:
            raise TypeError(f"unknown curriculum arguments: {sorted(unknown)}")
        kw.update(overrides)
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_curriculum_enable(self.handle, float(kw["initial_threshold"]),
                                                 float(kw["max_threshold"]), float(kw["threshold_increment"]),
                                                 int(kw["max_episodes_per_maze"]),
                                                 int(bool(kw["terminate_on_threshold"])), self._stream()),
                    "pe_curriculum_enable")
        self.curriculum_variant = variant

    def disable_curriculum(self):
        C.check(C.lib().pe_curriculum_disable(self.handle), "pe_curriculum_disable")

    def get_curriculum(self):
        """(threshold f64[n], counters i32[n,4]: episodes, successes, episodes on maze, flags)."""
        thr = torch.empty(self.num_envs, dtype=torch.float64, device=self.device)
        cnt = torch.empty((self.num_envs, 4), dtype=torch.int32, device=self.device)
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_curriculum_get(self.handle, _ptr(thr), _ptr(cnt), self._stream()),
                    "pe_curriculum_get")
        return thr, cnt

    def seed(self, seed, reset_episode_counters=True):
        with torch.cuda.device(self.device):
            C.check(C.lib().pe_seed(self.handle, int(seed) & 0xFFFFFFFFFFFFFFFF, int(bool(reset_episode_counters)),
                                    self._stream()), "pe_seed")
        self.cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
