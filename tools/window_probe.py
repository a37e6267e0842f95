#!/usr/bin/env python3
"""One driver-shaped window (20 steps after a 5-step warm-up graph) of the headline step per
process, with bench.py's preamble switched piece by piece:
  python tools/window_probe.py [upload=0|1] [episodes=0|1] [episodes_before=0|1] [idle_ms=0]
prints one JSON line (wall and HIP-event us per step of the first replay of the 20-step graph)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
sys.path.insert(0, REPO)


def main():
    opt = dict(a.split("=") for a in sys.argv[1:])
    upload, eps, idle_ms = int(opt.get("upload", 1)), int(opt.get("episodes", 1)), float(opt.get("idle_ms", 0))
    eps_before = int(opt.get("episodes_before", 0))  # the counter read before the warm-up instead
    import torch
    import bench
    from plantos_amd import PlantOSBatch
    n, K, W = 65536, 20, 5
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0")
    T = 64
    acts = torch.empty((T, n), dtype=torch.int32, device="cuda:0")
    for t in range(T):
        b.synth_actions(0, t, out=acts[t])

    def capture(steps):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(steps):
                b.step(acts[k % T])
        if upload:
            bench.upload_graph(torch, g)
        torch.cuda.synchronize()
        return g

    g20 = capture(K)
    g5 = capture(W)
    if eps_before:
        bench.episodes(b)
        torch.cuda.synchronize()
    g5.replay()
    torch.cuda.synchronize()
    if eps:
        bench.episodes(b)
    if idle_ms:
        time.sleep(idle_ms / 1e3)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    t0 = time.perf_counter()
    g20.replay()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(json.dumps({"upload": upload, "episodes": eps, "episodes_before": eps_before, "idle_ms": idle_ms, "wall_us_per_step": wall / K * 1e6,
                      "events_us_per_step": ev0.elapsed_time(ev1) / K * 1e3}), flush=True)


if __name__ == "__main__":
    main()
