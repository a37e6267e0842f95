#!/usr/bin/env python3
"""Per-step kernel time after pe_create (diagnostic, GPU): HIP events around each of
the first 60 steps at the headline shape, then again after 300 steps and after a
reset() (which refills every prefetched record).  Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402


def curve(b, acts, k):
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
    torch.cuda.synchronize()
    ev[0].record(st)
    for t in range(k):
        b.step(acts[t % len(acts)])
        ev[t + 1].record(st)
    torch.cuda.synchronize()
    return [round(ev[t].elapsed_time(ev[t + 1]) * 1e3, 2) for t in range(k)]


def main():
    n = 65536
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0")
    acts = [b.synth_actions(0, t) for t in range(64)]
    out = {"after_create": curve(b, acts, 60)}
    curve(b, acts, 300)
    out["steady"] = curve(b, acts, 30)
    b.reset()
    out["after_reset"] = curve(b, acts, 40)
    print(json.dumps(out), flush=True)
    b.close()


if __name__ == "__main__":
    main()
