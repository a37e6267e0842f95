"""bench.py's multi-GPU launcher on the CPU (no GPU work): `--gpus N` run directly
starts N ranks through torch.distributed.run before anything touches a GPU, the
ranks see world size N and reduce their timings with max; without N visible GPUs
it refuses with a non-zero status instead of benchmarking one GPU."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("OMP_NUM_THREADS", "1")
    return env


def test_launcher_starts_n_ranks_gloo():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--selftest"], capture_output=True, text=True,
                       timeout=240, env=_env(), cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["selftest"] is True
    assert lines[0]["max_over_ranks"] == 2.0  # max over ranks 0, 1 of rank + 1
    g = lines[0]["gather"]  # config 5's gather leg, same object shape as a GPU run's
    assert lines[0]["gather_order_ok"] is True
    assert g["bytes_gathered_per_step"] == 2 * g["bytes_per_rank_per_step"] == 2 * (4 * 64 * 107 + 6 * 64)
    assert g["root_ingress_bytes_per_step"] == g["bytes_per_rank_per_step"]
    for k in ("value", "us_per_step", "root_ingress_GBps", "steps", "launch", "collective"):
        assert k in g
    assert "gather" in g["collective"]


def test_graph_plan_and_launch_label():
    """the driver's short window (--steps 20) is one captured graph, long windows replay
    graphs aligned to the prefetch cadence, and the line's launch label says what the
    timed loop executed"""
    sys.path.insert(0, REPO)
    import bench
    assert bench.plan_graph(20, 64, 256) == 20  # the driver's window: one 20-step graph
    assert bench.plan_graph(20, 64, 256, "direct") == 0
    assert bench.launch_label(20, 0) == "20 direct host launches (one pe_step per step)"
    assert bench.plan_graph(153000, 64, 256) == 256
    assert bench.launch_label(1000, 256) == "hipGraph: 3 replays of 256 captured pe_step launches + 232 direct host launches"
    assert bench.launch_label(20, 20) == "hipGraph: 1 replay of 20 captured pe_step launches"
    assert bench.plan_graph(300, 64, 0) == 64
    assert bench.plan_graph(300, 512, 256) == 300
    assert bench.plan_graph(100000, 0, 256) == 0


def test_too_few_gpus_is_an_error():
    import torch
    if torch.cuda.device_count() >= 64:
        return
    r = subprocess.run([sys.executable, BENCH, "--gpus", "64"], capture_output=True, text=True, timeout=120,
                       env=_env(), cwd=REPO)
    assert r.returncode != 0
    assert "needs 64 visible GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
