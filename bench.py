#!/usr/bin/env python3
"""Benchmark of the batched PlantOSEnv step (BASELINE.json headline).

A "step" = one pe_step launch over the whole batch: every env consumes one
action and materializes obs f32[5C+27], reward f32, terminated u8, truncated u8
in HBM, auto-resetting (device-rng map generation) when done.  Inputs are
resident in HBM before the timed region; actions come from a pre-generated
device buffer of synthetic actions philox(seed, env, t) % 5 (4 B read per env-step).

  python bench.py [--gpus N --steps K --warmup W --envs E --grid G --rays C --range R]

--gpus N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set)
this process is one rank; run directly, it starts the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and
exits with their status -- or exits non-zero at once if fewer than N GPUs are
visible.  Each rank owns a disjoint shard of E envs (global ids rank*E ...), no
collective on the data path ("scaling": "weak"); barrier + max-over-ranks
timing.  --gather adds the host-boundary RCCL gather of each step's packed
(obs, reward, terminated, truncated) buffer to rank 0, pipelined behind the next
step (plantos_amd/shard.py step_gather).

After the headline window the same batch is timed again with desynchronized
episodes (every env at its own step count: ~n/1000 auto-resets in every step, the
steady state of a long training run); that result is the line's "desync" object.
"""
import argparse
import hashlib
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "rl-env_amd"))

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
    # >= 1e10 env-steps timed after a 1000-step warm-up (153000 x 65536 envs ~ 1.5 s)
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
    p.add_argument("--gather", action="store_true",
                   help="RCCL gather of each step's (obs, reward, done) to rank 0, pipelined")
    p.add_argument("--graph", type=int, default=64,
                   help="capture this many consecutive steps in one hipGraph and replay it (0: one host "
                        "launch per step); every captured step is a full pe_step launch")
    p.add_argument("--desync", action="store_true",
                   help="time the desynchronized episode mix as the headline window (default: synchronized "
                        "fresh episodes, desync as the secondary 'desync' object)")
    p.add_argument("--desync-steps", type=int, default=20000,
                   help="steps of the secondary desynchronized window (0: skip it)")
    p.add_argument("--prefetch-every", type=int, default=None,
                   help="steps between prefetched-reset launches (pe_config.prefetch_every; default: the library's)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--selftest", action="store_true",
                   help="launcher / rank plumbing only: gloo on the CPU, no GPU work (tests)")
    return p.parse_args()


# ---------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args):
    """Start args.gpus ranks with torch.distributed.run in a CHILD process (nothing
    here has touched the GPU: torch.cuda.device_count() does not initialize it) and
    return its exit status; rank 0 prints the JSON line."""
    if not args.selftest:
        import torch
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {visible}", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------- baselines / profiles
def cpu_baseline(args, plants, obstacles):
    """Oracle (C port of plantos_env.py step/reset) on the host cores this process
    may run on: same geometry, same synthetic-action workload, bounded sample
    (~cpu-seconds)."""
    sys.path.insert(0, REPO)
    from oracle import oracle as O

    threads = len(os.sched_getaffinity(0))
    cfg = O.config(args.grid, plants, obstacles, args.range, args.rays)
    n_envs = min(args.envs, 65536)
    steps = 20
    for _ in range(3):  # calibrate on the run itself until it lasts about cpu-seconds
        secs, _ = O.bench(cfg, n_envs, steps, args.seed, threads)
        if secs >= 0.7 * args.cpu_seconds or steps >= 20000:
            break
        steps = int(max(steps + 1, min(20000, steps * args.cpu_seconds / max(secs, 1e-6))))
    return {"value": n_envs * steps / secs, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n_envs} envs x {steps} steps ({secs:.1f} s) of the same synthetic workload, "
                      f"oracle/plantos_oracle.c, OpenMP {threads} threads (all cores in this process's "
                      f"affinity mask) on {cpu_model()}"}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def lib_sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()[:16]


def measured_traffic(cfg, sha):
    """Per-launch HBM bytes of this kernel/config from the committed rocprofv3 PMC
    summaries (profiles/pmc*_*.json, tools/pmc_summary.py), ONLY from a profile of
    this exact library (lib_sha of the .so the bench loaded).  traffic = 2 x
    FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts half the bytes of wide
    coalesced reads, MI355X_MICROARCH.md §HBM); the raw sum is kept beside it."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc*_*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        c = d.get("config", {})
        keys = ("envs_per_gpu", "grid", "rays", "lidar_range", "kernel")
        if d.get("lib_sha") == sha and all(c.get(k) == cfg.get(k) for k in keys):
            best = (p, d)
    if best is None:
        return None
    p, d = best
    return {"traffic": d["traffic_hi"], "traffic_raw": d["traffic"], "source": os.path.relpath(p, REPO)}


# ---------------------------------------------------------------- timed windows
def timed(torch, dist, device, K, one_step, chunk, graph, finish=None):
    """K steps bracketed by barrier + synchronize; (wall s, kernel ms per step).
    finish(): work of the K steps still queued elsewhere (pipelined gathers)."""
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)  # HIP events on the stream pe_step launches on
    if graph is not None:
        for _ in range(K // chunk):
            graph.replay()
        for k in range(K % chunk):
            one_step(k)
    else:
        for k in range(K):
            one_step(k)
    if finish is not None:
        finish()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / K
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def desynchronize(torch, b, seed):
    from plantos_amd import _capi as CA
    st = b.get_state()
    sc = st["scalars"]
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    sc[:, CA.PE_S_STEP] = torch.randint(0, 1000, (b.num_envs,), generator=g, dtype=torch.int32).to(sc.device)
    b.set_state(scalars=sc)


def selftest_rank(args, world, rank):
    """--selftest: the rank plumbing on the CPU (gloo): world size, barrier,
    max-over-ranks reduction, one line from rank 0.  No GPU work, no value."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": world,
                          "selftest": True, "max_over_ranks": float(t[0])}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.selftest:
        selftest_rank(args, world, rank)
        return

    import torch
    dist = None
    nccl_version = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"world size {dist.get_world_size()} != --gpus {args.gpus}")
        try:
            nccl_version = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:  # noqa: BLE001
            nccl_version = "unknown"
    device = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(device)

    from plantos_amd import PlantOSBatch, _capi
    from plantos_amd.shard import ShardedPlantOS

    G, C, R = args.grid, args.rays, args.range
    plants = args.plants if args.plants is not None else (10 if G <= 32 else 100)
    obstacles = args.obstacles if args.obstacles is not None else (12 if G <= 32 else 120)
    n = args.envs
    # rank r owns global env ids [r*n, (r+1)*n) (env_id_offset), no data-path collective
    shard = ShardedPlantOS(n, seed=args.seed, batch_factory=lambda n_, **kw: PlantOSBatch(
        n_, grid_size=G, num_plants=plants, num_obstacles=obstacles, lidar_range=R, lidar_channels=C,
        device=device, prefetch_every=args.prefetch_every, **kw))
    b = shard.batch
    if args.desync:
        desynchronize(torch, b, args.seed)
    T = args.action_steps
    actions = torch.empty((T, n), dtype=torch.int32, device=device)
    for t in range(T):
        b.synth_actions(args.seed, t, out=actions[t])
    gather = args.gather and world > 1

    def one_step(t):
        if gather:
            shard.step_gather(actions[t % T])  # RCCL gather of (obs, reward, term, trunc), pipelined
        else:
            b.step(actions[t % T])

    for t in range(args.warmup):
        one_step(t)
    shard.flush()
    torch.cuda.synchronize()
    K = args.steps
    # graph mode: one graph = `chunk` consecutive pe_step launches; step k of a replay
    # reads action row k % T (plain mode: step t reads row t % T).  K = reps * chunk + rest.
    chunk = min(args.graph, K) if (args.graph > 1 and not gather) else 0
    pf = b.prefetch_every
    if chunk > 1 and pf > 0 and chunk % pf:  # every replay must hold the same share of prefetch launches
        chunk = min(chunk * pf // math.gcd(chunk, pf), max(K, pf))
    graph = None
    if chunk > 1:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for k in range(chunk):
                b.step(actions[k % T])
        torch.cuda.synchronize()

    # with --gather the last gathers are part of the job: waited for inside the window
    elapsed, kern_ms = timed(torch, dist, device, K, one_step, chunk, graph, shard.flush if gather else None)
    b.raise_on_errors()
    total_steps = n * K * world
    value = total_steps / elapsed
    B = algorithmic_bytes(C, R)
    achieved = B * n / (kern_ms * 1e-3) / 1e9  # GB/s of ONE launch (one GPU's shard)

    desync = None
    if args.desync_steps > 0 and not args.desync:
        desynchronize(torch, b, args.seed)
        Kd = args.desync_steps
        for t in range(200):
            one_step(t)
        shard.flush()
        torch.cuda.synchronize()
        d_el, d_kms = timed(torch, dist, device, Kd, one_step, chunk, graph, shard.flush if gather else None)
        d_ach = B * n / (d_kms * 1e-3) / 1e9
        desync = {"value": n * Kd * world / d_el, "unit": "env-steps/s", "steps": Kd,
                  "us_per_step": d_el / Kd * 1e6, "kernel_us": d_kms * 1e3, "achieved": d_ach,
                  "frac": d_ach / HBM_PEAK_GBPS,
                  "note": "every env at its own step count in [0, 1000): ~n/1000 auto-resets per step"}
        b.raise_on_errors()
    if rank == 0:
        sha = lib_sha(_capi.LIB_PATH)
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
                       "parallelism": f"env-shard x{world}" + (" + rccl gather (pipelined)" if gather else ""),
                       "kernel": b.kernel_name,
                       "launch": f"hipGraph replay, {chunk} pe_step launches per graph" if graph is not None
                       else "one host launch per step"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                         "bytes_per_env_step": B, "kernel_ms": kern_ms},
            "lib_sha": sha,
        }
        if world > 1:
            out["config"]["rccl"] = nccl_version
        tr = measured_traffic(out["config"], sha)
        if tr is not None:
            out["roofline"].update({"traffic": tr["traffic"], "traffic_raw": tr["traffic_raw"],
                                    "traffic_source": tr["source"], "traffic_per_env_step": tr["traffic"] / n})
        else:
            out["roofline"]["traffic_note"] = f"no committed PMC profile of this library (lib_sha {sha})"
        if desync is not None:
            out["desync"] = desync
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, plants, obstacles)
        print(json.dumps(out), flush=True)
    b.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
