#!/usr/bin/env python3
"""Same-process timing of the f32 step kernel and its byte-coded twin (pe_step_codes,
BASELINE config 5's step) at one geometry, synchronized and desynchronized episodes
(diagnostics, not the bench line).  HIP events around replays of captured 256-step
graphs; one JSON line.   usage: python tools/codes_probe.py [--envs N] [--grid G ...]
(PLANTOS_HIP_LIB=... selects another build for same-box A/B)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402
import bench  # noqa: E402


def graph_us(b, acts, io, steps=256, reps=8):
    T = acts.shape[0]

    def body():
        for k in range(steps):
            b.step(acts[k % T], io=io)
    return bench.event_us(torch, bench.capture_graph(torch, body), reps, steps)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--grid", type=int, default=20)
    p.add_argument("--rays", type=int, default=16)
    p.add_argument("--range", type=int, default=6)
    p.add_argument("--plants", type=int, default=10)
    p.add_argument("--obstacles", type=int, default=12)
    a = p.parse_args()
    n, dev = a.envs, torch.device("cuda:0")
    res = {"envs": n, "grid": a.grid, "rays": a.rays, "range": a.range}
    for codes in (False, True):
        b = PlantOSBatch(n, grid_size=a.grid, num_plants=a.plants, num_obstacles=a.obstacles, lidar_range=a.range,
                         lidar_channels=a.rays, device=dev, obs_codes=codes)
        T = 64
        acts = torch.empty((T, n), dtype=torch.int32, device=dev)
        for t in range(T):
            b.synth_actions(0, t, out=acts[t])
        io = b.new_io()
        tag = "codes" if codes else "f32"
        for t in range(20):
            b.step(acts[t % T], io=io)
        torch.cuda.synchronize()
        res[f"{tag}_kernel"] = b.kernel_name
        res[f"{tag}_sync_us"] = graph_us(b, acts, io, reps=2)  # 256 + 512 steps: no truncation yet
        bench.desynchronize(torch, b, 0)
        for t in range(1300):
            b.step(acts[t % T], io=io)
        torch.cuda.synchronize()
        res[f"{tag}_desync_us"] = graph_us(b, acts, io)
        b.raise_on_errors()
        b.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
