#!/usr/bin/env python3
"""Rate of the SB3 VecEnv face (PlantOSVecEnv.step) at the headline shape: the
PCIe-inclusive path (numpy actions in, numpy obs/rewards/dones out, as SB3's
DummyVecEnv hands them to the policy) and the zero-copy path (tensors=True).

  python tools/vecenv_rate.py [--envs 65536] [--steps 300]
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from plantos_amd import PlantOSVecEnv  # noqa: E402


def rate(env, acts, steps, warm=20):
    env.reset()
    for t in range(warm):
        env.step(acts[t % len(acts)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(steps):
        obs, rew, done, infos = env.step(acts[t % len(acts)])
    if isinstance(obs, torch.Tensor):
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return env.num_envs * steps / dt, dt / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    kw = dict(grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16, device="cuda:0")
    rng = np.random.default_rng(0)
    acts_np = [rng.integers(0, 5, a.envs, dtype=np.int64) for _ in range(16)]
    out = {"envs": a.envs, "steps": a.steps}
    env = PlantOSVecEnv(a.envs, **kw)
    out["numpy_env_steps_per_s"], out["numpy_ms_per_step"] = rate(env, acts_np, a.steps)
    env.close()
    env = PlantOSVecEnv(a.envs, host_buffers=2, **kw)
    out["pinned_ring_env_steps_per_s"], out["pinned_ring_ms_per_step"] = rate(env, acts_np, a.steps)
    env.close()
    env = PlantOSVecEnv(a.envs, tensors=True, **kw)
    acts_t = [torch.as_tensor(x, device="cuda:0") for x in acts_np]
    out["tensors_env_steps_per_s"], out["tensors_ms_per_step"] = rate(env, acts_t, a.steps)
    env.close()
    out["obs_bytes_per_step"] = a.envs * (5 * 16 + 27) * 4
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
