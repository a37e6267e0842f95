#!/usr/bin/env python3
"""The driver-shaped short window (20 steps after a synchronize) under several launch
plans (diagnostic, GPU): one 20-step graph, a direct first step then a 19-step graph,
4 replays of a 5-step graph, 2 replays of a 10-step graph, 20 direct launches -- each
timed like bench.py's timed() (events on the launch stream, wall clock), alternating,
after a shared warm-up.  Prints one JSON line per plan with the per-step times."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402


def main():
    n, K = 65536, 20
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0")
    acts = torch.empty((64, n), dtype=torch.int32, device="cuda:0")
    for t in range(64):
        b.synth_actions(0, t, out=acts[t])

    def graph(steps):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(steps):
                b.step(acts[k % 64])
        torch.cuda.synchronize()
        return g

    g20, g19, g10, g5 = graph(20), graph(19), graph(10), graph(5)
    plans = {
        "graph20": lambda: g20.replay(),
        "direct1+graph19": lambda: (b.step(acts[0]), g19.replay()),
        "graph5x4": lambda: [g5.replay() for _ in range(4)],
        "graph10x2": lambda: [g10.replay() for _ in range(2)],
        "direct20": lambda: [b.step(acts[k]) for k in range(K)],
    }
    for k in range(5):
        b.step(acts[k])
    res = {p: {"events_us": [], "wall_us": []} for p in plans}
    stream = torch.cuda.current_stream()
    for rnd in range(6):
        for p, f in plans.items():
            for k in range(5):  # the bench's warm-up shape: a few direct steps, then a synchronize
                b.step(acts[k])
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            t0 = time.perf_counter()
            f()
            ev1.record(stream)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            if rnd:  # the first round warms every plan
                res[p]["events_us"].append(round(ev0.elapsed_time(ev1) / K * 1e3, 2))
                res[p]["wall_us"].append(round(wall / K * 1e6, 2))
    for p, r in res.items():
        print(json.dumps({"plan": p, **r}), flush=True)
    b.close()


if __name__ == "__main__":
    main()
