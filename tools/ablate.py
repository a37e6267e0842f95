#!/usr/bin/env python3
"""Phase ablation of the quadrant step kernel (diagnostics; outputs are WRONG
in the ablated builds, only their timings mean something).

  python tools/ablate.py build            # CPU: builds build/ablate/libplantos_hip_<bits>.so
  python tools/ablate.py run [--envs N]   # GPU: times every build, prints one JSON line

bits: 1 = no obs tile store, 2 = no ray-march, 4 = no round-2 window loads,
8 = no state commit.  Each build is timed in a fresh subprocess with HIP events
on torch's stream over 500 steps after 100 warm-up steps.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "rl-env_amd", "csrc", "plantos_batch.hip")
OUT = os.path.join(REPO, "build", "ablate")
VARIANTS = [0, 1, 2, 4, 8, 3, 7, 15]


def build():
    os.makedirs(OUT, exist_ok=True)
    for b in VARIANTS:
        so = os.path.join(OUT, f"libplantos_hip_{b}.so")
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               f"-DPE_ABLATE={b}", "-o", so, SRC]
        subprocess.run(cmd, check=True)
        print(so)


CHILD = r"""
import sys, json, torch
sys.path.insert(0, sys.argv[1])
from plantos_amd import PlantOSBatch
n = int(sys.argv[2])
b = PlantOSBatch(n, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16, device="cuda:0")
acts = torch.empty((64, n), dtype=torch.int32, device="cuda:0")
for t in range(64):
    b.synth_actions(0, t, out=acts[t])
for t in range(100):
    b.step(acts[t % 64])
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for t in range(512):
    b.step(acts[t % 64])
e.record()
torch.cuda.synchronize()
plain = s.elapsed_time(e) / 512
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for t in range(64):
        b.step(acts[t])
torch.cuda.synchronize()
s.record()
for r in range(8):
    g.replay()
e.record()
torch.cuda.synchronize()
print(json.dumps({"kernel": b.kernel_name, "ms": plain, "graph_ms": s.elapsed_time(e) / 512}))
"""


def run(n):
    res = {}
    for b in VARIANTS:
        env = dict(os.environ, PLANTOS_HIP_LIB=os.path.join(OUT, f"libplantos_hip_{b}.so"))
        out = subprocess.run([sys.executable, "-c", CHILD, os.path.join(REPO, "rl-env_amd"), str(n)], env=env,
                             capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            res[b] = {"error": out.stderr[-400:]}
            break
        res[b] = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps({"envs": n, "ablation_ms": res}))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        n = int(sys.argv[sys.argv.index("--envs") + 1]) if "--envs" in sys.argv else 65536
        run(n)
