#!/usr/bin/env python3
"""Where a batched MCTS search spends its cycles (diagnostics build, -DPE_MCTS_PROF).

  python tools/mcts_prof.py build        # CPU: build/mctsprof/libplantos_hip.so
  python tools/mcts_prof.py run          # GPU: 65536 envs, 50 sims x depth 100

Prints shader-clock cycles per simulation, averaged over lanes: tree phase
(selection + expansion), rollout, backprop + undo, and the RNG top-ups inside
them (per search)."""
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "build", "mctsprof", "libplantos_hip.so")


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    c = os.path.join(REPO, "rl-env_amd", "csrc")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DPE_MCTS_PROF", "-o", OUT, os.path.join(c, "plantos_batch.hip"), os.path.join(c, "pe_mcts.hip"),
                    os.path.join(c, "pe_pystream.cpp")], check=True)
    print(OUT)


def run():
    os.environ["PLANTOS_HIP_LIB"] = OUT
    sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
    import numpy as np
    import torch
    from plantos_amd import PlantOSBatch, _capi
    from plantos_amd.mcts import MCTS
    n = 65536
    b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                     device="cuda:0", seed=5)
    acts = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(37):
        b.step(b.synth_actions(5, t, out=acts))
    m = MCTS(b, n_simulations=50, max_depth=100, seed=123)
    m.search()
    torch.cuda.synchronize()
    L = _capi.lib()
    L.pe_mcts_debug_prof.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    buf = np.zeros(n * 4, np.uint64)
    _capi.check(L.pe_mcts_debug_prof(buf.ctypes.data_as(ctypes.c_void_p), buf.size), "prof")
    p = buf.reshape(n, 4).astype(np.float64)
    sims = 50
    print(json.dumps({"cycles_per_sim": {"tree": p[:, 0].mean() / sims, "rollout": p[:, 1].mean() / sims,
                                          "backprop_undo": p[:, 2].mean() / sims},
                      "topup_cycles_per_search": p[:, 3].mean(),
                      "rollout_cycles_per_step": p[:, 1].mean() / sims / 100}))


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
