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


def _paths():
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (repo, os.path.join(repo, "rl-env_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)


def _shard(n, codes):
    """this rank's ShardedPlantOS over an oracle-backed batch (global ids)"""
    _paths()
    from oracle_rollout import OracleBatch, OracleVec
    from plantos_amd.shard import ShardedPlantOS
    G, P, O_, R, C = CFG

    class ShardBatch(OracleBatch):
        def __init__(self, n_, env_id_offset, seed, obs_codes=False):
            super().__init__(n_, G, P, O_, R, C, seed=seed, max_steps=25, obs_codes=obs_codes)
            # re-key the shard to its GLOBAL env ids (env_id_offset semantics)
            ids = np.arange(env_id_offset, env_id_offset + n_)
            self.ov = OracleVec(self.cfg_t, ids, seed, max_steps=25)
            self.obs = torch.as_tensor(self.ov.obs())

    return ShardedPlantOS(n, seed=9, batch_factory=lambda n_, **kw: ShardBatch(n_, **kw), codes=codes)


def _drive(sh, rank, world, n, steps, pipelined):
    """step the shard `steps` times with global random actions; rank 0 checks every
    gathered global batch against ONE oracle batch over all world*n envs"""
    _paths()
    from oracle_rollout import OracleVec
    from plantos_amd.shard import shard_range
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
            last = [x.clone() for x in sh.unpack(sh.gathered(prev))]
            ok &= check(last)
            # gather_outputs after step_gather gathers the slot the last step wrote
        g = sh.gather_outputs()
        if rank == 0:
            ok &= bool((g[0] == last[0]).all())
    if rank == 0:
        ok &= not expect
    return ok


def _worker(rank, world, port, n, steps, q, pipelined=False, codes=False):
    """pipelined: step t+1's gather is issued before step t's result is checked (only
    step t's slot is waited for), so two gathers are in flight at once."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ok = _drive(_shard(n, codes), rank, world, n, steps, pipelined)
        if rank == 0:
            q.put(ok)
    finally:
        dist.destroy_process_group()


def _run(pipelined, world=2, codes=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 6, 40, q, pipelined, codes)) for r in range(world)]
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
    """world 1 with a process group (a torchrun job of one): every gather is a gloo
    gather of the rank to itself; gathered(slot) is the gather buffer (never an
    uninitialized one) and gather_outputs returns the latest step's"""
    _run(True, world=1)
    _run(False, world=1)


def test_two_rank_codes_gather_equals_one_batch():
    """codes=True: each rank moves its obs as byte codes (5C+27 B per env), the root
    expands the gathered [W, io_bytes] buffer once -- bit-equal to one oracle batch,
    plain and pipelined"""
    _run(False, codes=True)
    _run(True, codes=True)


def test_single_rank_codes_gather():
    _run(True, world=1, codes=True)


def test_no_process_group():
    """without torch.distributed initialized no collective runs at all: gathered(slot)
    is the slot itself ([1, io_bytes]), gather_outputs unpacks the batch's own io --
    checked against the oracle in both forms"""
    assert not dist.is_initialized()
    for codes in (False, True):
        for pipelined in (False, True):
            sh = _shard(6, codes)
            assert not sh._coll
            assert _drive(sh, 0, 1, 6, 30, pipelined)
            if pipelined:
                k = sh.step_gather(torch.zeros(6, dtype=torch.int64))
                assert sh.gathered(k).data_ptr() == sh._slots[k].data_ptr()


def test_codes_follow_the_batch_and_unpack_owns_nothing():
    """the shard's unpack layout follows the batch it built (a factory that writes codes
    regardless of `codes=`), obs_codes in cfg is refused, and a code-mode unpack returns
    fresh tensors (a later unpack never overwrites an earlier result) unless `out` is
    passed -- the same ownership as the f32 path's concatenation"""
    _paths()
    import pytest
    from plantos_amd.shard import ShardedPlantOS
    assert not dist.is_initialized()
    sh = _shard(6, False)
    base = sh.batch.__class__
    forced = ShardedPlantOS(6, seed=9, batch_factory=lambda n_, **kw: base(n_, **dict(kw, obs_codes=True)))
    assert forced.codes and forced.batch.obs_codes
    with pytest.raises(TypeError):
        ShardedPlantOS(6, seed=9, batch_factory=lambda n_, **kw: base(n_, **kw), obs_codes=True)
    sh = _shard(6, True)
    k = sh.step_gather(torch.zeros(6, dtype=torch.int64))
    first = sh.unpack(sh.gathered(k))
    keep = [x.clone() for x in first]
    k2 = sh.step_gather(torch.full((6,), 4, dtype=torch.int64))
    second = sh.unpack(sh.gathered(k2))
    assert all(a.data_ptr() != b.data_ptr() for a, b in zip(first, second))
    assert all(torch.equal(a, b) for a, b in zip(first, keep))
    out = sh.new_outputs()
    res = sh.unpack(sh.gathered(k2), out=out)
    assert all(r is o for r, o in zip(res, out)) and all(torch.equal(a, b) for a, b in zip(res, second))


def test_code_roundtrip_on_oracle_obs():
    """codes.py: expand(encode(obs)) == obs bit for bit over oracle rollouts of two
    geometries (incl. auto-reset obs), and the code io layout is 16-B padded"""
    _paths()
    from oracle_rollout import OracleVec
    from plantos_amd.codes import code_table, encode_obs, io_layout
    for cfg in (CFG, (20, 10, 12, 6, 16)):
        G, _, _, R, C = cfg
        ov = OracleVec(cfg, np.arange(16), 3, max_steps=30)
        t = code_table(G, R)
        rng = np.random.default_rng(1)
        for _ in range(40):
            obs = ov.step(rng.integers(0, 5, 16))[0]
            assert np.array_equal(t[encode_obs(obs, G, C, R)], obs)
        for n in (1, 6, 7, 65536):
            ro, to, tro, tot = io_layout(n, 5 * C + 27)
            assert ro % 16 == 0 and tot % 16 == 0 and tot >= tro + n

