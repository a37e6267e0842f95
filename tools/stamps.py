#!/usr/bin/env python3
"""Phase timeline of the sector step kernel from in-kernel s_memrealtime stamps
(diagnostics; the stamped build is a separate library, its run time is not a
bench number -- read the SHARES and the timeline shape, not the length).

  python tools/stamps.py build                 # CPU: build/stamps/libplantos_hip_stamps.so
  python tools/stamps.py run [--grid 20 --rays 16 --envs 65536]   # GPU

Stamps (lane 0 of each wave, 100 MHz = 10 ns ticks):
  0 entry  1 round-1 data in  2 round-2 loads landed + LDS written  3 after barrier
  4 rays/slice/commit done  5 after barrier_or  6 tile stores issued  7 stores drained
"""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(REPO, "build", "stamps", "libplantos_hip_stamps.so")
NAMES = ["entry", "round1", "round2+lds", "barrier", "compute", "barrier_or", "store_issue", "store_drain"]


def build(ablate=0):
    so = SO if not ablate else SO.replace(".so", f"_abl{ablate}.so")
    os.makedirs(os.path.dirname(so), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DPE_STAMPS", "-DPE_DEBUG_KNOBS", f"-DPE_ABLATE={ablate}", "-o", so,
                    os.path.join(REPO, "rl-env_amd", "csrc", "plantos_batch.hip")], check=True)
    print(so)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def run(argv):
    abl = int(argv[argv.index("--ablate") + 1]) if "--ablate" in argv else 0
    os.environ["PLANTOS_HIP_LIB"] = SO if not abl else SO.replace(".so", f"_abl{abl}.so")
    sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
    import numpy as np
    import torch
    from plantos_amd import PlantOSBatch
    from plantos_amd import _capi

    def arg(name, default):
        return int(argv[argv.index(name) + 1]) if name in argv else default

    G, C, n = arg("--grid", 20), arg("--rays", 16), arg("--envs", 65536)
    P, O = (10, 12) if G <= 32 else (100, 120)
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=O, lidar_range=6, lidar_channels=C,
                     device="cuda:0")
    acts = torch.empty((64, n), dtype=torch.int32, device="cuda:0")
    for t in range(64):
        b.synth_actions(0, t, out=acts[t])
    for t in range(300):
        b.step(acts[t % 64])
    torch.cuda.synchronize()
    b.step(acts[7])
    torch.cuda.synchronize()
    L = _capi.lib()
    L.pe_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    nw = (n + 63) // 64 * (int(os.environ.get("PE_QUAD_WAVES", "8")))
    buf = np.zeros(nw * 8, np.uint64)
    _capi.check(L.pe_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size), "stamps")
    st = buf.reshape(nw, 8).astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st - t0) * 10  # ns
    out = {"kernel": b.kernel_name, "envs": n, "waves": nw,
           "span_ns": int(rel[:, 7].max()),
           "abs_ns": {NAMES[k]: {"p0": int(rel[:, k].min()), "p50": int(np.median(rel[:, k])),
                                  "p100": int(rel[:, k].max())} for k in range(8)},
           "phase_ns": {f"{NAMES[k - 1]}->{NAMES[k]}": {"p50": int(np.median(rel[:, k] - rel[:, k - 1])),
                                                         "p90": int(np.percentile(rel[:, k] - rel[:, k - 1], 90))}
                        for k in range(1, 8)}}
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    else:
        run(sys.argv[2:])
