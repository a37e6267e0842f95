#!/usr/bin/env python3
"""Diagnostic (args: G P O R C n; default the g64 desync test): the first steps, state compared with the oracle
before and after each step (which env, which field first differs)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import oracle as O  # noqa: E402
from oracle_rollout import OracleVec  # noqa: E402
from plantos_amd import PlantOSBatch  # noqa: E402


def np_(t):
    return t.detach().cpu().numpy()


def cmp(tag, b, ov):
    st = b.get_state()
    for k, ref in (("cells", ov.b.cells), ("visits", ov.b.visits), ("scalars", ov.b.scal)):
        g = np_(st[k])
        bad = np.nonzero((g.reshape(len(g), -1) != ref.reshape(len(ref), -1)).any(1))[0]
        print(tag, k, "mismatching envs:", bad[:10].tolist(), len(bad))
        if len(bad) and k == "scalars":
            print("  gpu", g[bad[0]].tolist(), "ref", ref[bad[0]].tolist())


cfg = tuple(int(v) for v in sys.argv[1:6]) if len(sys.argv) > 5 else (64, 100, 120, 6, 64)
G, P, Ob, R, C = cfg
n = int(sys.argv[6]) if len(sys.argv) > 6 else 192
b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C, seed=31,
                 device="cuda:0")
print("kernel", b.kernel_name)
ov = OracleVec(cfg, np.arange(n), 31)
cmp("create", b, ov)
rng = np.random.default_rng(5)
start = (999 - rng.integers(0, 40, n)).astype(np.int32)
sc = np_(b.get_state()["scalars"])
sc[:, O.S_STEP] = start
b.set_state(scalars=sc)
ov.b.scal[:, O.S_STEP] = start
cmp("set_state", b, ov)
act = torch.empty(n, dtype=torch.int32, device="cuda:0")
for t in range(3):
    b.synth_actions(31, t, out=act)
    a_np = np_(act)
    obs, rew, te, tr = b.step(act)
    o = ov.step(a_np)
    bad = np.nonzero(np_(rew) != o[1].astype(np.float32))[0]
    print("step", t, "reward mismatches", bad[:10].tolist(), [(int(a_np[k]), float(np_(rew)[k]), float(o[1][k])) for k in bad[:5]])
    cmp(f"step{t}", b, ov)
