"""Multi-rank path on CPU (world_size 2, gloo, 127.0.0.1): each rank steps its
shard (global ids rank*n ...) through plantos_amd.shard with an oracle-backed
batch; the gathered global batch on rank 0 must equal ONE oracle batch over all
2n envs, step after step, through the auto-reset."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

CFG = (7, 3, 3, 3, 12)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, steps, q, pipelined=False):
    """pipelined: step t+1's gather is issued before step t's result is checked (only
    step t's slot is waited for), so two gathers are in flight at once."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "rl-env_amd"), here):
        sys.path.insert(0, p)
    from oracle_rollout import OracleBatch, OracleVec
    from plantos_amd.shard import ShardedPlantOS, shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G, P, O_, R, C = CFG

        class ShardBatch(OracleBatch):
            def __init__(self, n_, env_id_offset, seed):
                super().__init__(n_, G, P, O_, R, C, seed=seed, max_steps=25)
                # re-key the shard to its GLOBAL env ids (env_id_offset semantics)
                ids = np.arange(env_id_offset, env_id_offset + n_)
                self.ov = OracleVec(self.cfg_t, ids, seed, max_steps=25)
                self.obs = torch.as_tensor(self.ov.obs())

        sh = ShardedPlantOS(n, seed=9, batch_factory=lambda n_, **kw: ShardBatch(n_, **kw))
        assert shard_range(rank, world, n) == (rank * n, (rank + 1) * n)
        full = OracleVec(CFG, np.arange(world * n), 9, max_steps=25) if rank == 0 else None
        rng = np.random.default_rng(0)
        ok = True
        expect = []  # rank 0: the single-batch oracle's outputs of steps not checked yet

        def check(g):
            obs, rew, te, tr = expect.pop(0)
            good = bool((g[0].numpy() == obs).all() and (g[1].numpy() == rew.astype(np.float32)).all())
            return good and bool((g[2].numpy().astype(bool) == te).all() and (g[3].numpy().astype(bool) == tr).all())

        prev = None
        for t in range(steps):
            a_glob = torch.as_tensor(rng.integers(0, 5, world * n))
            a_loc = sh.scatter_actions(a_glob if rank == 0 else None)
            assert (a_loc.numpy() == a_glob.numpy()[rank * n:(rank + 1) * n]).all()
            if rank == 0:
                expect.append(full.step(a_glob.numpy())[:4])
            if pipelined:
                k = sh.step_gather(a_loc)
                if prev is not None:  # step t-1's gather: waited for while step t's is in flight
                    sh.wait(prev)
                    if rank == 0:
                        ok &= check(sh.unpack(sh.gathered(prev)))
                prev = k
            else:
                sh.step(a_loc)
                g = sh.gather_outputs()
                if rank == 0:
                    ok &= check(g)
                else:
                    assert g is None
        if pipelined:
            sh.flush()
            if rank == 0:
                ok &= check(sh.unpack(sh.gathered(prev)))
                # gather_outputs after step_gather gathers the slot the last step wrote
            g = sh.gather_outputs()
            if rank == 0:
                ok &= bool((g[0] == sh.unpack(sh.gathered(prev))[0]).all())
        if rank == 0:
            ok &= not expect
            q.put(ok)
    finally:
        dist.destroy_process_group()


def _run(pipelined, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 6, 40, q, pipelined)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_two_rank_shards_equal_one_batch():
    """one packed gather per step (gather_outputs)"""
    _run(False)


def test_pipelined_step_gather_equals_one_batch():
    """step_gather: double-buffered outputs, each step's gather issued asynchronously
    and waited for only before its buffer is written again (flush at the end)"""
    _run(True)


def test_single_rank_step_gather_and_gather_outputs():
    """world 1: step_gather issues no collective; gathered(slot) is the slot itself
    (never an uninitialized buffer) and gather_outputs returns the latest step's"""
    _run(True, world=1)
    _run(False, world=1)
