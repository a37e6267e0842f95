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
timing.  `value` is that replica throughput.  Every run then also times the
host-boundary leg of BASELINE config 5 ("with RCCL gather"): each step's packed
(obs, reward, terminated, truncated) buffer gathered to rank 0 over RCCL,
pipelined behind the next step (plantos_amd/shard.py step_gather) -- the line's
"gather" object (with one rank there is nothing to gather and it says so).

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
    p.add_argument("--gather-steps", type=int, default=500,
                   help="steps of the gather-every-step leg (RCCL gather of each step's outputs to rank 0, "
                        "pipelined; the line's 'gather' object; 0: skip it)")
    p.add_argument("--graph", type=int, default=64,
                   help="capture up to this many consecutive steps in one hipGraph and replay it (0: one host "
                        "launch per step); every captured step is a full pe_step launch")
    p.add_argument("--short-window", choices=("graph", "direct"), default="graph",
                   help="a window of <= 256 steps: one captured graph of its steps after the warm-up steps as "
                        "one captured graph (graph), or one host launch per step (direct)")
    p.add_argument("--desync", action="store_true",
                   help="time the desynchronized episode mix as the headline window (default: synchronized "
                        "fresh episodes, desync as the secondary 'desync' object)")
    p.add_argument("--desync-steps", type=int, default=20000,
                   help="steps of the secondary desynchronized window (0: skip it)")
    p.add_argument("--desync-warmup", type=int, default=1300,
                   help="untimed steps between desynchronizing and the secondary window (>= max_steps + the "
                        "prefetch cadence: every env reset once and its next record generated)")
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
    this exact library (lib_sha of the .so the bench loaded).  traffic = FETCH_SIZE
    + WRITE_SIZE with the gfx950 x2 applied to the kernel's streamed reads only
    (MI355X_MICROARCH.md §HBM; calibrated on known byte counts of our access shapes,
    profiles/r3r_fetch_calibration.json: gathered 16-B rows are counted in full);
    the raw sum and the all-reads-x2 upper bound are kept beside it."""
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
    return {"traffic": d.get("traffic_cal", d["traffic_hi"]), "traffic_raw": d["traffic"],
            "traffic_hi": d["traffic_hi"], "source": os.path.relpath(p, REPO),
            "calibration": d.get("calibration")}


def _symbol_bytetile(sym):
    """True / False: the byte-coded obs tile of a pe_step_quad<C, R, ONEWORD, NW, BT, EPB>
    symbol (its BT template argument; pe_step_far always has it); None: not parseable."""
    import re
    if "pe_step_far<" in sym:
        return True
    m = re.search(r"pe_step_quad<\s*\d+,\s*\d+,\s*(?:true|false),\s*\d+,\s*(true|false)", sym)
    return None if m is None else m.group(1) == "true"


def rocprof_kernel_ns(cfg, sha):
    """The step kernel's average launch duration (ns) from the committed rocprofv3
    --kernel-trace --stats summaries of this exact library and config
    (profiles/kstats_*.json, tools/kstats_summary.py; or a PMC summary's stats_avg_ns),
    keyed like measured_traffic; None without one."""
    import glob
    best = None
    keys = ("envs_per_gpu", "grid", "rays", "lidar_range", "kernel")
    for p in sorted(glob.glob(os.path.join(REPO, "profiles", "kstats_*.json")) +
                    glob.glob(os.path.join(REPO, "profiles", "pmc*_*.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        c = d.get("config", {})
        ns = d.get("avg_ns", d.get("stats_avg_ns"))
        # the obs mode of the profiled kernel must be the benched one's: a byte-coded
        # (codes / byte-tile) symbol never stands for an f32-tile kernel or vice versa
        bt = _symbol_bytetile(d.get("kernel_symbol", ""))
        if bt is not None and bt != ("bytetile" in str(cfg.get("kernel", ""))):
            continue
        if ns and not d.get("desync") and d.get("lib_sha") == sha and all(c.get(k) == cfg.get(k) for k in keys):
            if best is None or os.path.basename(p).startswith("kstats_"):
                best = (p, float(ns))
    if best is None:
        return None
    return {"ns": best[1], "source": os.path.relpath(best[0], REPO)}


# ---------------------------------------------------------------- timed windows
def upload_graph(torch, gr):
    """hipGraphUpload the captured graph before the timed window (executes nothing):
    its first replay otherwise pays the upload, ~1 us per step of a 20-step window
    (profiles/r3g_window_first_replay.json).  Best effort: a runtime without it
    just uploads at the first replay."""
    import ctypes
    try:
        # the HIP runtime this process already has mapped (the one torch loaded): a
        # runtime opened by name could be another copy, whose hipGraphUpload would get a
        # graph-exec handle it does not own
        with open("/proc/self/maps") as f:
            paths = {ln.split()[-1] for ln in f if "libamdhip64.so" in ln and ln.split()[-1].startswith("/")}
        if len(paths) != 1:
            return False
        hip = ctypes.CDLL(paths.pop())
        exe = gr.raw_cuda_graph_exec()
        hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        return hip.hipGraphUpload(ctypes.c_void_p(exe), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    except (OSError, AttributeError, IndexError, RuntimeError):
        return False


DIRECT_MAX = 256  # windows of at most this many steps: the short-window plan (see plan_graph)


def plan_graph(K, graph_max, pf, short="graph"):
    """Steps per captured graph for a K-step window (0: direct launches).  A short
    window (K <= DIRECT_MAX, e.g. the driver's 20 steps) is ONE K-step graph, captured
    and uploaded before the warm-up (itself one W-step graph, see main): host launches cost 7-14 us per
    pe_step in the first tens of calls after a synchronize (profiles/r4j_host_cost.json),
    above the ~9.6 us kernel, so a direct-launch window times the host (same box,
    alternating runs, profiles/r4l_drv_ab.jsonl: direct 12.8-14.3 us per step, one graph
    11.6-13.2, 5-step graphs warmed by the warm-up 11.8-13.1).  short="direct": direct
    launches.  A longer window replays a graph whose length is a multiple of the
    prefetch cadence pf (every replay then holds the same share of prefetch launches),
    the rest as direct launches."""
    if graph_max <= 1:
        return 0
    if K <= DIRECT_MAX:
        return K if short == "graph" else 0
    if K <= graph_max:
        return K
    chunk = graph_max
    if pf > 0 and chunk % pf:
        chunk = chunk * pf // math.gcd(chunk, pf)
    return min(chunk, K)


def launch_label(K, chunk):
    """What the timed loop of timed() executes for K steps and this chunk."""
    if not chunk:
        return f"{K} direct host launches (one pe_step per step)"
    reps, rest = K // chunk, K % chunk
    lab = f"hipGraph: {reps} replay{'s' if reps != 1 else ''} of {chunk} captured pe_step launches"
    return lab + (f" + {rest} direct host launches" if rest else "")


def timed(torch, dist, device, K, one_step, chunk, graph, finish=None):
    """K steps bracketed by barrier + synchronize; (wall s, kernel ms per step).
    finish(): work of the K steps still queued elsewhere (pipelined gathers).
    device None: the CPU plumbing of --selftest (no events; kernel ms = wall)."""
    if device is None:
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(K):
            one_step(k)
        if finish is not None:
            finish()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t[0])
        return elapsed, elapsed / K * 1e3
    if dist:
        dist.barrier(group=BARRIER_GROUP)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(device)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # HIP events on the stream pe_step launches on; the opening one is recorded before
    # the wall clock starts (its host-side cost, ~10 us on ROCm, is instrumentation)
    ev0.record(stream)
    t0 = time.perf_counter()
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
    elapsed = time.perf_counter() - t0  # this rank's K steps; the job's time is the max over ranks
    if dist:
        dist.barrier(group=BARRIER_GROUP)
        torch.cuda.synchronize()
    kern_ms = ev0.elapsed_time(ev1) / K
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def episodes(b):
    """per-env episode counters (every auto-reset increments one)"""
    import torch
    from plantos_amd import _capi as CA
    return b.get_state(parts=("scalars",))["scalars"][:, CA.PE_S_EPISODE].to(torch.int64)


def resets_since(torch, dist, b, ep0):
    """auto-resets performed by all ranks since the counters ep0 were read (outside any
    timed window: one state read before and one after)"""
    r = (episodes(b) - ep0).sum().reshape(1).to(torch.int64)
    if dist:
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
    return int(r.item())


def desynchronize(torch, b, seed):
    from plantos_amd import _capi as CA
    st = b.get_state()
    sc = st["scalars"]
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    sc[:, CA.PE_S_STEP] = torch.randint(0, 1000, (b.num_envs,), generator=g, dtype=torch.int32).to(sc.device)
    b.set_state(scalars=sc)


class GatherLoop:
    """One step of BASELINE config 5's host boundary on every rank: the shard steps
    into one of two output slots and its packed outputs go to rank 0 (RCCL gather,
    async); rank 0 then turns the PREVIOUS step's gathered slot into the global
    (obs f32 [W*n, D], reward, terminated, truncated) -- with a codes shard one
    expansion kernel over the [W, io_bytes] gather buffer, into output tensors the
    consumer owns and reuses -- i.e. what a consumer of the global batch pays,
    inside the timed window."""

    def __init__(self, shard, actions, rank):
        self.shard, self.actions, self.root = shard, actions, rank == 0
        self.prev = None
        self.out = shard.new_outputs() if (shard.codes and self.root) else None

    def step(self, t):
        sh = self.shard
        k = sh.step_gather(self.actions[t % self.actions.shape[0]])
        if self.prev is not None:
            self._consume(self.prev)
        self.prev = k

    def _consume(self, k):
        sh = self.shard
        sh.wait(k)  # (the stream waits for the collective; the host does not)
        if self.root:
            sh.unpack(sh.gathered(k), out=self.out)

    def finish(self):
        if self.prev is not None:
            self._consume(self.prev)
            self.prev = None
        self.shard.flush()


def capture_graph(torch, body):
    """body() captured into one hipGraph (executes nothing), uploaded, returned."""
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        body()
    upload_graph(torch, gr)
    torch.cuda.synchronize()
    return gr


def event_us(torch, gr, reps, per):
    """HIP events around `reps` replays of graph gr (after one untimed replay): us per
    unit, `per` units per replay."""
    stream = torch.cuda.current_stream()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        gr.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * per)


def gather_leg(torch, dist, device, shard, Kg, loop, world):
    """BASELINE config 5's host-boundary leg: Kg steps of `loop` (GatherLoop): each
    step's packed outputs gathered to rank 0 (RCCL over xGMI; gloo in --selftest),
    pipelined behind the next step, and unpacked there.  With a process group: host
    launches -- an RCCL collective inside a captured graph is not exercised on the
    one-GPU boxes this code is tested on, and a hang there would cost the whole scaling
    run.  Without one (one rank, nothing to gather): the Kg (step into a slot + the
    previous slot's expansion) pairs as ONE captured graph, as the headline window."""
    for t in range(20):
        loop.step(t)
    loop.finish()
    if device is not None:
        torch.cuda.synchronize()
    graph, chunk = None, 0
    parts = {}
    if dist is None and device is not None:
        def body():
            for t in range(Kg):
                loop.step(t)
            loop.finish()
        graph, chunk = capture_graph(torch, body), Kg
        graph.replay()  # (the first replay of a graph is the slow one)
        torch.cuda.synchronize()
        # the two kernels of a step apart (HIP events over graphs of 64 of each): what the
        # leg's step costs beyond them is launch gap
        sh = shard
        acts = loop.actions

        def steps_only():
            for t in range(64):
                sh.step_gather(acts[t % acts.shape[0]])
        if loop.out is not None:
            def expands_only():
                for t in range(64):
                    sh.unpack(sh.gathered(t & 1), out=loop.out)
            parts["expand_us"] = event_us(torch, capture_graph(torch, expands_only), 4, 64)
            # the root's expansion at W = 8 ranks (BASELINE config 5): 8 copies of the slot in
            # one [8, io_bytes] buffer -> the global f32 outputs of 8 x n envs, one launch
            W8 = 8
            src8 = sh.gathered(0).reshape(1, -1).repeat(W8, 1)
            out8 = sh.new_outputs(W8)

            def expands_w8():
                for t in range(16):
                    sh.unpack(src8, out=out8)
            parts["expand_w8_us"] = event_us(torch, capture_graph(torch, expands_w8), 4, 16)
            parts["expand_w8_bytes"] = {"read": int(src8.numel()),
                                        "written": int(sum(t.numel() * t.element_size() for t in out8))}
            del src8, out8
        parts["step_us"] = event_us(torch, capture_graph(torch, steps_only), 4, 64)
        if "expand_w8_us" in parts:
            parts["root_step_w8_us"] = parts["step_us"] + parts["expand_w8_us"]
            parts["root_step_w8_note"] = ("implied per-step root cost at 8 ranks: its own codes step + the expansion "
                                          "of 8 gathered blocks (the RCCL ingress overlaps both)")
    g_el, g_kms = timed(torch, dist, device, Kg, loop.step, chunk, graph, None if graph is not None else loop.finish)
    n = shard.n
    per_rank = shard.io_bytes()
    us = g_el / Kg * 1e6
    backend = "RCCL (nccl backend)" if device is not None else "gloo (selftest)"
    D = shard.batch.obs_dim
    launch = (f"hipGraph: one replay of {Kg} captured (pe_step_codes into a slot + pe_expand_obs_codes of the "
              f"previous slot) pairs (no process group: nothing to gather)" if graph is not None else
              f"{Kg} direct host launches, each step's gather issued async (double-buffered), the previous step's "
              f"gathered slot unpacked on rank 0")
    return {"value": n * Kg * world / g_el, "unit": "env-steps/s", "steps": Kg, "us_per_step": us,
            "kernel_us_per_step": g_kms * 1e3, "codes": bool(shard.codes), **parts,
            "payload": ("obs as byte codes (5C+27 B/env) + reward f32 + terminated u8 + truncated u8, expanded "
                        "on rank 0 by one pe_expand_obs_codes launch into contiguous f32 outputs"
                        if shard.codes else "obs f32 + reward f32 + terminated u8 + truncated u8; rank 0 "
                        "concatenates the ranks' parts"),
            "bytes_per_rank_per_step": per_rank, "bytes_gathered_per_step": per_rank * world,
            "f32_bytes_per_rank_per_step": 4 * n * D + 6 * n,
            "root_ingress_bytes_per_step": per_rank * (world - 1),
            "root_ingress_GBps": per_rank * (world - 1) / (us * 1e-6) / 1e9,
            "root_expanded_bytes_per_step": (4 * D + 6) * n * world,
            "launch": launch,
            "collective": (f"torch.distributed.gather over {backend} to rank 0" + (" (one rank: to itself)" if world == 1
                                                                                     else "")
                           if dist else "none: one rank, nothing to gather (the step into the slot buffers only)")}


class _SelftestBatch:
    """--selftest stand-in for PlantOSBatch on the CPU: the io-buffer interface only,
    outputs = the global env id (plumbing of the shard / gather leg; no env work)."""

    def __init__(self, n, env_id_offset=0, seed=0, obs_dim=107):
        import torch
        self.torch, self.num_envs, self.obs_dim, self.device = torch, n, obs_dim, torch.device("cpu")
        self.ids = torch.arange(env_id_offset, env_id_offset + n, dtype=torch.float32)

    def io_bytes(self):
        return 4 * self.num_envs * self.obs_dim + 6 * self.num_envs

    def new_io(self):
        return self.torch.zeros(self.io_bytes(), dtype=self.torch.uint8)

    def io_views(self, io):
        n, D = self.num_envs, self.obs_dim
        f32 = self.torch.float32
        return (io[:4 * n * D].view(f32).view(n, D), io[4 * n * D:4 * n * (D + 1)].view(f32),
                io[4 * n * (D + 1):4 * n * (D + 1) + n], io[4 * n * (D + 1) + n:])

    def step(self, actions, io=None):
        n, D = self.num_envs, self.obs_dim
        io[:4 * n * D].view(self.torch.float32).view(n, D).copy_(self.ids[:, None])

    def close(self):
        pass


def selftest_rank(args, world, rank):
    """--selftest: the rank plumbing on the CPU (gloo): world size, barrier,
    max-over-ranks reduction, the gather leg's collective and its object, one line
    from rank 0.  No GPU work, no value."""
    import torch
    import torch.distributed as dist
    from plantos_amd.shard import ShardedPlantOS
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = 64
    shard = ShardedPlantOS(n, batch_factory=lambda n_, **kw: _SelftestBatch(n_, **kw))
    acts = torch.zeros((1, n), dtype=torch.int64)
    gather = gather_leg(torch, dist if world > 1 else None, None, shard, 10, GatherLoop(shard, acts, rank), world)
    ok = True
    if rank == 0:  # every rank's slot arrived, in global env order
        obs = shard.unpack(shard.gathered(0))[0]
        ok = bool((obs[:, 0] == torch.arange(world * n, dtype=torch.float32)).all())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "env-steps/s", "n_gpus": world,
                          "selftest": True, "max_over_ranks": float(t[0]), "gather": gather,
                          "gather_order_ok": ok}), flush=True)
    if world > 1:
        dist.destroy_process_group()


WAIT_FLAGS = {"spin": 1, "yield": 2, "blocking": 4}  # hipDeviceSchedule*
# the process group of the barriers around the timed windows (main: PLANTOS_BARRIER)
BARRIER_GROUP = None


def set_wait_policy(torch, local):
    """How the host waits for the GPU's completions (the window's closing synchronize):
    PLANTOS_WAIT=auto (HIP's default, untouched) | spin | yield | blocking
    (hipSetDeviceFlags on this rank's device, before anything else initialises it) |
    poll (HSA_ENABLE_INTERRUPT=0: completion signals polled, not interrupt-driven).
    Returns the policy applied."""
    pol = os.environ.get("PLANTOS_WAIT", "auto")
    if pol == "poll":
        os.environ["HSA_ENABLE_INTERRUPT"] = "0"
    elif pol in WAIT_FLAGS:
        import ctypes
        # the HIP runtime torch loaded (its own copy; the step library binds the same one)
        hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        if hip.hipSetDevice(local) != 0 or hip.hipSetDeviceFlags(WAIT_FLAGS[pol]) != 0:
            raise SystemExit(f"bench.py: hipSetDeviceFlags({pol}) failed")
    elif pol != "auto":
        raise SystemExit(f"bench.py: PLANTOS_WAIT={pol}: auto | spin | yield | blocking | poll")
    return pol


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
    wait_policy = set_wait_policy(torch, local)
    dist = None
    nccl_version = None
    # a process group whenever a launcher started this process (WORLD_SIZE set) -- also
    # for one rank, so a torchrun job of one runs the same RCCL path (init, barriers,
    # max-over-ranks, the gather leg) as the 8-GPU job
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"world size {dist.get_world_size()} != --gpus {args.gpus}")
        # the windows' barriers: RCCL (PLANTOS_BARRIER=nccl, an all-reduce kernel on the GPU
        # right before the window) or a host-side gloo group over the same rendezvous (gloo)
        barrier_kind = os.environ.get("PLANTOS_BARRIER", "nccl")
        if barrier_kind == "gloo":
            global BARRIER_GROUP
            BARRIER_GROUP = dist.new_group(backend="gloo")
        elif barrier_kind != "nccl":
            raise SystemExit(f"bench.py: PLANTOS_BARRIER={barrier_kind}: nccl | gloo")
        try:
            nccl_version = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception:  # noqa: BLE001
            nccl_version = "unknown"
    device = torch.device("cuda", local if dist else 0)
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
    def one_step(t):
        b.step(actions[t % T])


    def capture(steps):
        if not steps:
            return None
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for k in range(steps):
                b.step(actions[k % T])
        upload_graph(torch, gr)
        torch.cuda.synchronize()
        return gr

    K = args.steps
    # graph mode: one graph = `chunk` consecutive pe_step launches; step k of a replay
    # reads action row k % T (plain mode: step t reads row t % T).  K = reps * chunk + rest.
    # Captured (nothing executes) BEFORE the warm-up, so that the warm-up steps run
    # right up to the timed window: a GPU left idle while the host captures starts the
    # window below its clocks (driver-shaped 20-step windows: ~1 us per step)
    pf = b.prefetch_every
    chunk = plan_graph(K, args.graph, pf, args.short_window)
    graph = capture(chunk)
    # the short window's W warm-up steps as one captured W-step graph: the first graph replay
    # of a process pays more than later ones, so the window's is not the first
    # (profiles/r4aa_drv_ab.jsonl: 11.2 us per step median vs 12.1 with direct warm-up steps)
    wgraph = capture(args.warmup) if chunk and K <= DIRECT_MAX and args.warmup > 0 else None
    # the auto-reset counters are read before the warm-up (PLANTOS_EP0=warmup, the default) and
    # the line counts the resets of warm-up + window: read between the warm-up and the window
    # (PLANTOS_EP0=window, exact window count) the state read -- a kernel, a copy, a host sync --
    # costs a driver-shaped 20-step window ~1 us per step (profiles/r6/window_probe_r6v.jsonl)
    ep_at = os.environ.get("PLANTOS_EP0", "warmup")
    if ep_at not in ("warmup", "window"):
        raise SystemExit(f"bench.py: PLANTOS_EP0={ep_at}: warmup | window")
    if ep_at == "warmup":
        ep0 = episodes(b)
        torch.cuda.synchronize()
    if wgraph is not None:
        wgraph.replay()
    else:
        for t in range(args.warmup):
            one_step(t)
    torch.cuda.synchronize()
    if ep_at == "window":
        ep0 = episodes(b)
    elapsed, kern_ms = timed(torch, dist, device, K, one_step, chunk, graph)
    b.raise_on_errors()
    resets = resets_since(torch, dist, b, ep0)
    total_steps = n * K * world
    value = total_steps / elapsed
    B = algorithmic_bytes(C, R)
    achieved_window = B * n / (kern_ms * 1e-3) / 1e9  # GB/s of ONE launch (one GPU's shard), timed window
    # the step kernel's launch duration back to back, live: HIP events over >= 2048 steps of
    # captured graphs after the timed window (a short window's events also hold the gap
    # before its first graph node: 20 steps 11.7 us against 9.45 us per kernel, r4)
    ev_chunk = chunk if chunk >= 256 else 256
    ev_graph = graph if ev_chunk == chunk else capture(ev_chunk)
    kern_us_events = event_us(torch, ev_graph, max(1, 2048 // ev_chunk), ev_chunk)
    if dist:
        t = torch.tensor([kern_us_events], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        kern_us_events = float(t[0])
    b.raise_on_errors()

    desync = None
    if args.desync_steps > 0 and not args.desync:
        desynchronize(torch, b, args.seed)
        Kd = args.desync_steps
        d_chunk = plan_graph(Kd, args.graph, pf)
        d_graph = graph if d_chunk == chunk else capture(d_chunk)
        # warm-up: every env resets once (max_steps) and its record is regenerated (one
        # prefetch cadence) -- the steady state of a desynchronized run.  The synchronized
        # window before left the records stale (a batch truncating together resets in
        # place, consuming none), and a 200-step warm-up timed ~5 % of the window's resets
        # as in-place map generations (11.3 vs 10.95 us per step, r4h)
        for t in range(args.desync_warmup):
            one_step(t)
        torch.cuda.synchronize()
        dep0 = episodes(b)
        d_el, d_kms = timed(torch, dist, device, Kd, one_step, d_chunk, d_graph)
        d_ach = B * n / (d_kms * 1e-3) / 1e9
        desync = {"value": n * Kd * world / d_el, "unit": "env-steps/s", "steps": Kd,
                  "resets_in_window": resets_since(torch, dist, b, dep0),
                  "us_per_step": d_el / Kd * 1e6, "kernel_us": d_kms * 1e3, "achieved": d_ach,
                  "frac": d_ach / HBM_PEAK_GBPS, "launch": launch_label(Kd, d_chunk),
                  "note": "every env at its own step count in [0, 1000): ~n/1000 auto-resets per step"}
        b.raise_on_errors()

    # BASELINE config 5's host-boundary leg (gather_leg)
    gather = None
    if args.gather_steps > 0:
        # its own shard (same global ids) whose step keeps the obs as byte codes where the
        # geometry has a byte-coded sector kernel (config 5's 20x20 / 16 rays does)
        try:
            gsh = ShardedPlantOS(n, seed=args.seed, codes=True, batch_factory=lambda n_, **kw: PlantOSBatch(
                n_, grid_size=G, num_plants=plants, num_obstacles=obstacles, lidar_range=R, lidar_channels=C,
                device=device, prefetch_every=args.prefetch_every, **kw))
        except ValueError:
            gsh = shard
        if gsh is not shard:
            desynchronize(torch, gsh.batch, args.seed)
        # what actually ran: the codes shard is desynchronized above; the headline shard
        # only if the timed (--desync) or the secondary desync window desynchronized it
        desynced = gsh is not shard or args.desync or desync is not None
        gather = gather_leg(torch, dist, device, gsh, args.gather_steps, GatherLoop(gsh, actions, rank), world)
        gather["episodes"] = "desynchronized" if desynced else "synchronized (fresh episodes)"
        gather["kernel"] = gsh.batch.kernel_name
        if gsh.codes:
            gather["expand_kernel"] = "pe_expand_codes_kernel"
        gsh.batch.raise_on_errors()
        if gsh is not shard:
            gsh.close()
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
                       "parallelism": f"env-shard x{world} (independent replicas; RCCL gather leg: 'gather')",
                       "kernel": b.kernel_name,
                       "launch": launch_label(K, chunk) + (f" (warm-up: one {args.warmup}-step graph)"
                                                           if K <= DIRECT_MAX and chunk and args.warmup > 0 else ""),
                       "host_wait": wait_policy,
                       "barrier": (os.environ.get("PLANTOS_BARRIER", "nccl") if dist else None)},
            ("resets_in_window" if ep_at == "window" else "resets_in_warmup_and_window"): resets,
            "lib_sha": sha,
        }
        # roofline of the step kernel: algorithmic bytes x envs / its average launch
        # duration measured live in THIS run (HIP events on the launch stream around >= 2048
        # back-to-back graph-replayed steps); the committed rocprofv3 stats of this library
        # and config are a cross-check only, flagged when they disagree by more than 5 %
        rp = rocprof_kernel_ns(out["config"], sha)
        k_us = kern_us_events
        achieved = B * n / (k_us * 1e-6) / 1e9
        rp_us = rp["ns"] / 1e3 if rp else None
        out["roofline"] = {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS, "traffic": None, "bytes_per_env_step": B,
            "kernel_us": k_us,
            "kernel_us_source": "HIP events, >= 2048 back-to-back steps of captured graphs (this run)",
            "kernel_us_rocprof": rp_us,
            "kernel_us_rocprof_source": (f"committed rocprofv3 --kernel-trace --stats average of this library and "
                                         f"config ({rp['source']})" if rp else None),
            "rocprof_agrees": (abs(k_us - rp_us) <= 0.05 * rp_us) if rp else None,
            "frac_rocprof": B * n / (rp_us * 1e-6) / 1e9 / HBM_PEAK_GBPS if rp else None,
            "kernel_us_events": kern_us_events,
            "frac_events": B * n / (kern_us_events * 1e-6) / 1e9 / HBM_PEAK_GBPS,
            "kernel_us_window": kern_ms * 1e3, "frac_window": achieved_window / HBM_PEAK_GBPS,
            "window_note": "kernel_us_window / frac_window: HIP events over the timed window itself (a short "
                           "window adds the launch of its first graph node)"}
        if dist:
            out["config"]["rccl"] = nccl_version
        tr = measured_traffic(out["config"], sha)
        if tr is not None:
            out["roofline"].update({"traffic": tr["traffic"], "traffic_raw": tr["traffic_raw"],
                                    "traffic_all_reads_x2": tr["traffic_hi"], "traffic_source": tr["source"],
                                    "traffic_calibration": tr["calibration"],
                                    "traffic_per_env_step": tr["traffic"] / n})
        else:
            out["roofline"]["traffic_note"] = f"no committed PMC profile of this library (lib_sha {sha})"
        if desync is not None:
            out["desync"] = desync
        if gather is not None:
            out["gather"] = gather
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, plants, obstacles)
        print(json.dumps(out), flush=True)
    b.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
