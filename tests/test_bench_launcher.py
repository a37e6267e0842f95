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


def test_too_few_gpus_is_an_error():
    import torch
    if torch.cuda.device_count() >= 64:
        return
    r = subprocess.run([sys.executable, BENCH, "--gpus", "64"], capture_output=True, text=True, timeout=120,
                       env=_env(), cwd=REPO)
    assert r.returncode != 0
    assert "needs 64 visible GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
