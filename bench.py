#!/usr/bin/env python3
"""Benchmark of the batched PlantOSEnv step (BASELINE.json headline).

A "step" = one pe_step launch over the whole batch: every env consumes one
action and materializes obs f32[5C+27], reward f32, terminated u8, truncated u8
in HBM, auto-resetting (device-rng map generation) when done.  Inputs are
resident in HBM before the timed region; actions come from a pre-generated
device buffer of synthetic actions philox(seed, env, t) % 5 (4 B read per env-step).

  python bench.py [--gpus N --steps K --warmup W --envs E --grid G --rays C --range R]

N>1: one process per GPU (torch.distributed.run); each rank owns a disjoint
shard of E envs (global ids rank*E ...), no collective on the data path
("scaling": "weak"); barrier + max-over-ranks timing.  --gather adds the
host-boundary RCCL gather of (obs, reward, done) to rank 0 every step.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))

import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "env-steps/sec at 64k parallel 20×20 envs; achieved HBM GB/s vs roofline"


def algorithmic_bytes(C, R):
    """B = B_io + B_state per env-step."""
    b_io = 4 + 4 * (5 * C + 27) + 4 + 2
    b_state = 8 + 50 + 2 + C * R + 16
    return b_io + b_state


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # >= 1e10 env-steps timed after a 1000-step warm-up (153000 x 65536 envs ~ 1.7 s)
    p.add_argument("--steps", type=int, default=153000)
    p.add_argument("--warmup", type=int, default=1000)
    p.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--grid", type=int, default=20)
    p.add_argument("--plants", type=int, default=None)
    p.add_argument("--obstacles", type=int, default=None)
    p.add_argument("--rays", type=int, default=16)
    p.add_argument("--range", type=int, default=6)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--action-steps", type=int, default=64, help="distinct pre-generated action rows")
    p.add_argument("--gather", action="store_true", help="RCCL gather of (obs,reward,done) to rank 0 each step")
    p.add_argument("--graph", type=int, default=64,
                   help="capture this many consecutive steps in one hipGraph and replay it (0: one host "
                        "launch per step); every captured step is a full pe_step launch")
    p.add_argument("--desync", action="store_true",
                   help="steady-state episode mix: env e starts at a random step count in [0, max_steps), so "
                        "about n/1000 envs auto-reset in every step (default: synchronized fresh episodes)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    return p.parse_args()


def cpu_baseline(args, plants, obstacles):
    """Oracle (C port of plantos_env.py step/reset) on the host cores: same
    geometry, same synthetic-action workload, bounded sample (~cpu-seconds)."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O

    threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    cfg = O.config(args.grid, plants, obstacles, args.range, args.rays)
    n_envs = min(args.envs, 65536)
    secs, _ = O.bench(cfg, n_envs, 10, args.seed, threads)  # calibration
    rate = n_envs * 10 / max(secs, 1e-6)
    steps = int(max(10, min(20000, args.cpu_seconds * rate / n_envs)))
    secs, _ = O.bench(cfg, n_envs, steps, args.seed, threads)
    return {"value": n_envs * steps / secs, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n_envs} envs x {steps} steps ({secs:.1f} s) of the same synthetic workload, "
                      f"oracle/plantos_oracle.c, OpenMP {threads} threads on {cpu_model()}"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def measured_traffic(cfg):
    """Per-launch HBM bytes of this kernel/config from the committed rocprofv3 PMC
    summaries (profiles/pmc_*.json, pmc64_*.json; tools/pmc_summary.py): FETCH_SIZE + WRITE_SIZE
    in bytes, collected in separate passes.  PMC cannot run inside the timed
    process, so the bench line cites the profile it took the number from."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc*_*.json"))):  # pmc_*, pmc64_*
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        c = d.get("config", {})
        keys = ("envs_per_gpu", "grid", "rays", "lidar_range", "kernel")
        if all(c.get(k) == cfg.get(k) for k in keys):
            best = (p, d)
    if best is None:
        return None, None, None
    p, d = best
    return d["traffic"], d.get("traffic_hi"), os.path.relpath(p, REPO)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(device)

    from plantos_amd import PlantOSBatch

    G, C, R = args.grid, args.rays, args.range
    plants = args.plants if args.plants is not None else (10 if G <= 32 else 100)
    obstacles = args.obstacles if args.obstacles is not None else (12 if G <= 32 else 120)
    n = args.envs
    from plantos_amd.shard import ShardedPlantOS

    # rank r owns global env ids [r*n, (r+1)*n) (env_id_offset), no data-path collective
    shard = ShardedPlantOS(n, seed=args.seed, batch_factory=lambda n_, **kw: PlantOSBatch(
        n_, grid_size=G, num_plants=plants, num_obstacles=obstacles, lidar_range=R, lidar_channels=C,
        device=device, **kw))
    b = shard.batch
    if args.desync:
        from plantos_amd import _capi as CA
        st = b.get_state()
        sc = st["scalars"]
        g = torch.Generator(device="cpu").manual_seed(args.seed + 1)
        sc[:, CA.PE_S_STEP] = torch.randint(0, 1000, (n,), generator=g, dtype=torch.int32).to(sc.device)
        b.set_state(scalars=sc)
    T = args.action_steps
    actions = torch.empty((T, n), dtype=torch.int32, device=device)
    for t in range(T):
        b.synth_actions(args.seed, t, out=actions[t])
    def one_step(t):
        b.step(actions[t % T])
        if args.gather and world > 1:
            shard.gather_outputs(root=0)  # RCCL gather of (obs, reward, term, trunc) to rank 0

    for t in range(args.warmup):
        one_step(t)
    torch.cuda.synchronize()
    K = args.steps
    # graph mode: one graph = `chunk` consecutive pe_step launches; step k of a replay
    # reads action row k % T (plain mode: step t reads row t % T).  K = reps * chunk + rest.
    chunk = min(args.graph, K) if (args.graph > 1 and not args.gather) else 0
    graph = None
    if chunk > 1:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for k in range(chunk):
                b.step(actions[k % T])
        torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        for k in range(K // chunk):
            graph.replay()
        for k in range(K % chunk):
            one_step(k)
    else:
        for k in range(K):
            one_step(args.warmup + k)
    ev1.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # average launch duration: HIP events on the launch stream over the timed region
    # (back-to-back launches, so this includes the ~1-2 us inter-kernel boundary)
    kern_ms = ev0.elapsed_time(ev1) / K
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    b.raise_on_errors()
    total_steps = n * K * world
    value = total_steps / elapsed
    B = algorithmic_bytes(C, R)
    achieved = B * n / (kern_ms * 1e-3) / 1e9  # GB/s of ONE launch (one GPU's shard)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32/f32",
            "data": "synthetic (device-rng maps, philox actions" + (", desynchronized episodes)" if args.desync
                                                                     else ")"),
            "config": {"workload": f"{n} envs/GPU, {G}x{G} grid, {C} rays, range {R}, {plants} plants, "
                                   f"{obstacles} obstacles, auto-reset, actions in HBM",
                       "envs_per_gpu": n, "grid": G, "rays": C, "lidar_range": R,
                       "parallelism": f"env-shard x{world}" + (" + rccl gather" if args.gather else ""),
                       "kernel": b.kernel_name,
                       "launch": f"hipGraph replay, {chunk} pe_step launches per graph" if graph is not None
                       else "one host launch per step"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                         "bytes_per_env_step": B, "kernel_ms": kern_ms},
        }
        tr, tr_hi, src = measured_traffic(out["config"])
        if tr is not None:
            out["roofline"].update({"traffic": tr, "traffic_fetch_x2": tr_hi, "traffic_source": src,
                                    "traffic_per_env_step": tr / n})
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, plants, obstacles)
        print(json.dumps(out), flush=True)
    b.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
