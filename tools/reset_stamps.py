#!/usr/bin/env python3
"""Stamps of the auto-reset path (diagnostic build -DPE_STAMPS_RESET): R0 enter,
R1 terminal copies, R2 terminal info, R3 map generated + written, R4 tile stored,
R5 fresh obs written.  Prints p50/p100 of each phase in ns."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PLANTOS_HIP_LIB"] = os.path.join(REPO, "build", "stamps", "libplantos_hip_rstamps.so")
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from plantos_amd import PlantOSBatch, _capi  # noqa: E402

n = 65536
b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16, device="cuda:0")
acts = torch.zeros(n, dtype=torch.int32, device="cuda:0") + 4
for t in range(1000):
    b.step(acts)
torch.cuda.synchronize()
L = _capi.lib()
L.pe_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64]
nw = n // 64 * 4
buf = np.zeros(nw * 8, np.uint64)
_capi.check(L.pe_debug_stamps(buf.ctypes.data_as(ctypes.c_void_p), buf.size), "stamps")
st = buf.reshape(nw, 8).astype(np.int64)
st = st[3::4]  # commit waves
out = {}
for k in range(1, 6):
    d = (st[:, k] - st[:, k - 1]) * 10
    out[f"R{k-1}->R{k}"] = {"p50": int(np.median(d)), "p100": int(d.max())}
out["span_R0_R5_p100"] = int((st[:, 5].max() - st[:, 0].min()) * 10)
print(json.dumps(out))
