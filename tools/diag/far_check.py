#!/usr/bin/env python3
"""Diagnose a step-kernel parity failure: n envs of one geometry, episodes
desynchronized (or not), `steps` steps vs the oracle over ALL envs; prints for the
first mismatching step the mismatching envs (block, lane, done flag) and which obs
indices differ (ray / field).   usage: python tools/diag/far_check.py G P O R C n steps [desync]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "rl-env_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
from oracle import oracle as O  # noqa: E402
from oracle_rollout import OracleVec  # noqa: E402
from plantos_amd import PlantOSBatch  # noqa: E402


def main():
    G, P, Ob, R, C, n, steps = (int(v) for v in sys.argv[1:8])
    desync = len(sys.argv) > 8 and sys.argv[8] == "1"
    seed = 5
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C, seed=seed,
                     device="cuda:0")
    ov = OracleVec((G, P, Ob, R, C), np.arange(n), seed)
    if desync:
        start = np.random.default_rng(11).integers(0, 1000, n).astype(np.int32)
        sc = b.get_state(parts=("scalars",))["scalars"].cpu().numpy()
        sc[:, O.S_STEP] = start
        b.set_state(scalars=sc)
        ov.b.scal[:, O.S_STEP] = start
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    out = {"kernel": b.kernel_name, "n": n, "desync": desync}
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        o_obs, o_rew, o_te, o_tr, *_ = ov.step(act.cpu().numpy())
        g = obs.cpu().numpy()
        bad = np.nonzero((g != o_obs).any(1))[0]
        rbad = np.nonzero(rew.cpu().numpy() != o_rew.astype(np.float32))[0]
        if len(bad) or len(rbad):
            done = o_te | o_tr
            recs = []
            for e in bad[:12]:
                idx = np.nonzero(g[e] != o_obs[e])[0]
                recs.append({"env": int(e), "block": int(e // 64), "lane": int(e % 64), "done": bool(done[e]),
                             "block_done": int(done[(e // 64) * 64:(e // 64) * 64 + 64].sum()),
                             "idx": idx[:20].tolist(), "rays": sorted(set((idx[idx < 5 * C] // 5).tolist()))[:20],
                             "gpu": g[e][idx[:6]].tolist(), "ref": o_obs[e][idx[:6]].tolist()})
            out.update({"step": t, "n_bad_obs": int(len(bad)), "n_bad_rew": int(len(rbad)),
                        "n_done": int(done.sum()), "bad_done": int(done[bad].sum()), "first": recs})
            break
    else:
        out["ok"] = True
    print(json.dumps(out))
    b.close()


if __name__ == "__main__":
    main()
