#!/usr/bin/env python3
"""Micro-benchmark of pe_step variants on one GPU (diagnostics, not the bench line).

Times, with HIP events on torch's stream:
  - plain steps (no env finishes),
  - the auto-reset step (every env truncates at max_steps),
  - a hipGraph-captured loop of steps (launch-gap-free throughput).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402


def timed(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--grid", type=int, default=20)
    p.add_argument("--rays", type=int, default=16)
    p.add_argument("--range", type=int, default=6)
    p.add_argument("--plants", type=int, default=10)
    p.add_argument("--obstacles", type=int, default=12)
    a = p.parse_args()
    n = a.envs
    b = PlantOSBatch(n, grid_size=a.grid, num_plants=a.plants, num_obstacles=a.obstacles, lidar_range=a.range,
                     lidar_channels=a.rays, seed=1, device="cuda:0", max_steps=1000)
    T = 64
    acts = torch.empty((T, n), dtype=torch.int32, device="cuda:0")
    for t in range(T):
        b.synth_actions(1, t, out=acts[t])
    it = [0]

    def step():
        b.step(acts[it[0] % T])
        it[0] += 1

    for _ in range(50):
        step()
    res = {"kernel": b.kernel_name, "envs": n}
    res["plain_ms"] = timed(step, 200)
    # advance to the step before truncation, then time the all-env reset step
    while it[0] < 999:
        step()
    torch.cuda.synchronize()
    res["reset_step_ms"] = timed(step, 1)
    # graph capture of 50 steps
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(50):
            b.step(acts[k % T])
    torch.cuda.synchronize()
    res["graph_ms_per_step"] = timed(g.replay, 20) / 50
    res["env_steps_per_s_graph"] = n / (res["graph_ms_per_step"] * 1e-3)
    res["env_steps_per_s_plain"] = n / (res["plain_ms"] * 1e-3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
