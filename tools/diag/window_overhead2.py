#!/usr/bin/env python3
"""Timed-window bracket variants (diagnostic, GPU): wall us of a 20-step graph replay
(headline shape) with the opening event recorded inside / outside the wall clock,
and with no events.  Prints one JSON line."""
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
    acts = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    for _ in range(50):
        b.step(acts)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            b.step(acts)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()

    def v_inside():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6, e0.elapsed_time(e1) * 1e3

    def v_outside():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(st)
        t0 = time.perf_counter()
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6, e0.elapsed_time(e1) * 1e3

    def v_none():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6, None

    out = {}
    for name, f in (("inside", v_inside), ("outside", v_outside), ("none", v_none)):
        r = sorted((f() for _ in range(40)), key=lambda x: x[0])
        out[name] = {"wall_us_p50": r[20][0], "event_us_p50": r[20][1], "wall_us_min": r[0][0]}
    print(json.dumps(out), flush=True)
    b.close()


if __name__ == "__main__":
    main()
