#!/usr/bin/env python3
"""Fixed cost of bench.py's timed window (diagnostic, GPU): wall time of the
barrier/synchronize/event bracket with 0..K pe_step launches inside, direct and
as one captured graph, at the headline shape.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0")
    acts = torch.zeros(n, dtype=torch.int32, device="cuda:0")
    for _ in range(50):
        b.step(acts)
    torch.cuda.synchronize()
    out = {}

    def med(f, reps=30):
        v = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f()
            v.append((time.perf_counter() - t0) * 1e6)
        v.sort()
        return v[len(v) // 2]

    out["sync_idle_us"] = med(torch.cuda.synchronize)
    ev = torch.cuda.Event(enable_timing=True)
    out["event_record_sync_us"] = med(lambda: (ev.record(), torch.cuda.synchronize()))
    for K in (1, 5, 20):
        out[f"direct_{K}_us"] = med(lambda: ([b.step(acts) for _ in range(K)], torch.cuda.synchronize()))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(K):
                b.step(acts)
        torch.cuda.synchronize()
        out[f"graph_{K}_us"] = med(lambda: (g.replay(), torch.cuda.synchronize()))
        t0 = time.perf_counter()
        g.replay()
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        out[f"graph_{K}_issue_us"] = t_issue * 1e6
    print(json.dumps(out), flush=True)
    b.close()


if __name__ == "__main__":
    main()
