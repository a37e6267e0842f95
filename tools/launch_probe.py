#!/usr/bin/env python3
"""Driver-shaped 20-step windows of the headline step (65536 envs, 20x20, 16 rays) launched
three ways, alternating: one replay of a captured 20-launch graph (bench.py's short window),
20 launches from a tight ctypes loop (arguments precomputed), and 20 PlantOSBatch.step calls.
Each window: synchronize, wall clock + HIP events around the launches, synchronize.
Prints one JSON line per window (GPU; diagnostics for bench.py's short-window plan)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))


def main():
    import torch
    from plantos_amd import PlantOSBatch
    n, K, W = 65536, 20, 5
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0")
    T = 64
    acts = torch.empty((T, n), dtype=torch.int32, device="cuda:0")
    for t in range(T):
        b.synth_actions(0, t, out=acts[t])
    stream = torch.cuda.current_stream()
    L, h = b._L, b.handle
    r, te, tr = b._out_ptrs
    e0, e1, e2 = b._ep_ptrs
    args = [(h, acts[k].data_ptr(), 4, b.obs.data_ptr(), r, te, tr, b._tobs_ptr, e0, e1, e2, stream.cuda_stream)
            for k in range(T)]

    def capture(steps):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(steps):
                b.step(acts[k % T])
        torch.cuda.synchronize()
        return g

    g20, g5 = capture(K), capture(W)
    for _ in range(50):
        b.step(acts[0])
    torch.cuda.synchronize()

    def window(mode):
        g5.replay()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        t0 = time.perf_counter()
        if mode == "graph":
            g20.replay()
        elif mode == "ctypes":
            st = L.pe_step
            for k in range(K):
                st(*args[k])
        else:
            for k in range(K):
                b.step(acts[k])
        t_issue = time.perf_counter() - t0
        ev1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return {"mode": mode, "wall_us_per_step": wall / K * 1e6, "events_us_per_step": ev0.elapsed_time(ev1) / K * 1e3,
                "host_issue_us": t_issue * 1e6}

    for r_ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
        for mode in ("graph", "ctypes", "step"):
            d = window(mode)
            d["round"] = r_
            print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
