#!/usr/bin/env python3
"""Host-side cost of one step launch (diagnostic, GPU): wall time of K back-to-back
PlantOSBatch.step() calls with the GPU kept busy, per call, vs the same K steps' GPU
time -- a driver-shaped short window of direct launches is host-bound when the first
exceeds the kernel time.  Also the pieces: torch's current-stream lookup, a bare
ctypes pe_step call.  Prints one JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import torch  # noqa: E402

from plantos_amd import PlantOSBatch  # noqa: E402


def main():
    n = 65536
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0")
    acts = [b.synth_actions(0, t) for t in range(64)]
    for t in range(200):
        b.step(acts[t % 64])
    torch.cuda.synchronize()
    out = {}
    for K in (20, 200):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        t0 = time.perf_counter()
        for t in range(K):
            b.step(acts[t % 64])
        t1 = time.perf_counter()
        ev1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[f"K{K}"] = {"host_us_per_call": (t1 - t0) / K * 1e6, "wall_us_per_step": (t2 - t0) / K * 1e6,
                        "gpu_us_per_step": ev0.elapsed_time(ev1) / K * 1e3}
    t0 = time.perf_counter()
    for _ in range(2000):
        torch.cuda.current_stream(0).cuda_stream
    out["current_stream_us"] = (time.perf_counter() - t0) / 2000 * 1e6
    L = b._L
    a = acts[0]
    s = torch.cuda.current_stream(0).cuda_stream
    r, te, tr = b._out_ptrs
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        L.pe_step(b.handle, a.data_ptr(), 4, b.obs.data_ptr(), r, te, tr, b._tobs_ptr, b._ep_ptrs[0], b._ep_ptrs[1],
                  b._ep_ptrs[2], s)
    out["bare_pe_step_us"] = (time.perf_counter() - t0) / 200 * 1e6
    torch.cuda.synchronize()
    out["kernel"] = b.kernel_name
    print(json.dumps(out), flush=True)
    b.close()


if __name__ == "__main__":
    main()
