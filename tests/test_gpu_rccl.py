"""bench.py's multi-rank path on the GPU (BASELINE config 5's code path): a
torch.distributed.run job of ONE rank -- the driver's launch line with
--nproc-per-node 1 -- initializes the RCCL (nccl backend) process group, times with
barriers and a max-over-ranks all_reduce, and runs the gather-every-step leg through
RCCL (the rank gathering to itself).  The 8-GPU job differs only in the world size
(one GPU per box here; two ranks cannot share one GPU under RCCL)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_torchrun_one_rank_rccl_bench_line():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--envs", "4096", "--steps", "40", "--warmup", "5", "--desync-steps", "0",
           "--gather-steps", "40", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = lines[0]
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["rccl"]
    g = d["gather"]
    assert "RCCL" in g["collective"] and g["value"] > 0 and g["bytes_gathered_per_step"] == g["bytes_per_rank_per_step"]
