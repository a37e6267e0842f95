#!/usr/bin/env python3
"""The driver's short window (diagnostic, GPU): 5 warm-up steps, then 20 timed steps
as bench.py times them, with the graph's FIRST replay, its second replay, and 20
direct launches -- wall vs event us per step.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402


def window(run, K):
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    t0 = time.perf_counter()
    run()
    e1.record(st)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e6, e0.elapsed_time(e1) / K * 1e3


def main():
    n, K = 65536, 20
    out = {}
    for trial in range(2):
        b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                         device="cuda:0")
        acts = torch.zeros(n, dtype=torch.int32, device="cuda:0")
        for _ in range(5):
            b.step(acts)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(K):
                b.step(acts)
        torch.cuda.synchronize()
        up = None
        if trial == 1:  # the bench's upload before the window
            import bench
            up = bench.upload_graph(torch, g)
            torch.cuda.synchronize()
        r = {"graph_first": window(g.replay, K), "graph_second": window(g.replay, K),
             "direct": window(lambda: [b.step(acts) for _ in range(K)], K),
             "graph_third": window(g.replay, K)}
        out[f"trial{trial}"] = {k: {"wall_us": v[0], "event_us": v[1]} for k, v in r.items()}
        out[f"trial{trial}"]["uploaded"] = up
        b.close()
        del g
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
