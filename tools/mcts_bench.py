#!/usr/bin/env python3
"""Batched MCTS benchmark: MCTS.search for every env at once.

  python tools/mcts_bench.py [--envs 65536 --grid 20 --sims 50 --depth 100 --reps 5]

One "search" is the reference's MCTS.search (mcts_custom_trainer.py:91-139) for one
env: n_sims simulations of up to max_depth + 1 sim-env steps each (train_mcts uses
n_sims 50, max_depth 100, :275).  Prints one JSON line: searches/s over all envs
(device, HIP events on the search stream, clone + search kernels), the nominal
sim-steps/s (n_sims * (max_depth + 1) per search), and the CPU baseline: the C
oracle (oracle/plantos_mcts.c) on a bounded sample of the same searches, one env
per host thread.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "rl-env_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--grid", type=int, default=20)
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--depth", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=256)
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()
    import numpy as np
    import torch
    from plantos_amd import PlantOSBatch
    from plantos_amd.mcts import MCTS

    G = args.grid
    P, O_, R, C = (10, 12, 6, 16) if G <= 32 else (100, 120, 6, 64)
    n = args.envs
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=O_, lidar_range=R, lidar_channels=C,
                     device="cuda:0", seed=5)
    acts = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(37):
        b.step(b.synth_actions(5, t, out=acts))
    m = MCTS(b, n_simulations=args.sims, max_depth=args.depth, seed=123)
    m.search()
    torch.cuda.synchronize()
    st = b.get_state()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = []
    for _ in range(args.reps):
        e0.record(s)
        m.search()
        e1.record(s)
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    avg = sum(ms) / len(ms)
    searches = n / (avg / 1e3)
    nominal = args.sims * (args.depth + 1)

    # CPU baseline: the oracle on a sample of the same searches
    from oracle import oracle as O
    cells, visits, expl, sc = (st[k].cpu().numpy() for k in ("cells", "visits", "explored", "scalars"))
    cfg = O.config(G, P, O_, R, C)
    k = min(args.cpu_sample, n)

    def one(e):
        r = O.NpMT(7 + e)
        return O.mcts_search(cfg, cells[e], visits[e], expl[e], sc[e], r, args.sims, 1.414, args.depth)[0]

    t0 = time.perf_counter()
    with ThreadPoolExecutor(args.cpu_threads) as ex:
        list(ex.map(one, range(k)))
    cpu_s = time.perf_counter() - t0
    print(json.dumps({
        "metric": "mcts_searches_per_s", "value": searches, "unit": "searches/s", "n_envs": n,
        "ms_per_search_batch": avg, "ms_reps": ms, "config": {"grid": G, "n_simulations": args.sims,
                                                                 "max_depth": args.depth, "c_param": 1.414},
        "nominal_sim_steps_per_s": searches * nominal,
        "cpu_baseline": {"value": k / cpu_s, "unit": "searches/s", "cores": args.cpu_threads, "kind": "port",
                         "sample": f"{k} searches (oracle/plantos_mcts.c, one env per thread)"},
    }))


if __name__ == "__main__":
    main()
