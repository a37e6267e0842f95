"""GPU parity of the byte-coded obs boundary (pe_config.obs_codes, pe_step_codes,
pe_expand_obs_codes; plantos_amd/codes.py): a code-mode batch expanded to f32 must
equal the oracle (and a plain f32 batch) bit for bit, every step, through
synchronized truncations (the lane-per-env reset path), desynchronized episodes
(cooperative resets from prefetched code records) and at 64x64 / 64 rays; the
expansion of many back-to-back buffers (a root's gather buffer) is one kernel; and
the sharded job's codes gather on one GPU (no process group) equals the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu

CFG = {"g20": (20, 10, 12, 6, 16), "g64": (64, 100, 120, 6, 64)}


def np_(t):
    return t.detach().cpu().numpy()


def make(cfg, n, **kw):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = cfg
    return PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                        device="cuda:0", **kw)


def test_code_table_matches_host():
    from plantos_amd.codes import code_table
    for name in CFG:
        b = make(CFG[name], 64, obs_codes=True)
        G, _, _, R, _ = CFG[name]
        assert np.array_equal(b.code_table(), code_table(G, R))
        b.close()


def test_codes_refused_without_byte_tile():
    """geometries without a byte-coded sector kernel refuse obs_codes (PE_ERR_ARG)"""
    with pytest.raises(ValueError):
        make((25, 10, 12, 6, 16), 64, obs_codes=True)


@pytest.mark.parametrize("name,n,steps,spread", [
    ("g20", 4096, 1010, None),   # every env truncates at step 1000 together: lane-per-env resets
    ("g20", 2048, 160, 150),     # desynchronized: prefetched (code) records, cooperative resets
    ("g64", 192, 50, 40),
    ("g20", 1000, 30, None),     # a ragged last block
])
def test_codes_equal_oracle(name, n, steps, spread):
    cfg = CFG[name]
    b = make(cfg, n, seed=13, obs_codes=True)
    assert b.obs_codes
    ov = OracleVec(cfg, np.arange(n), 13)
    if spread:
        rng = np.random.default_rng(5)
        start = (999 - rng.integers(0, spread, n)).astype(np.int32)
        sc = np_(b.get_state()["scalars"])
        sc[:, O.S_STEP] = start
        b.set_state(scalars=sc)
        ov.b.scal[:, O.S_STEP] = start
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    obs = torch.empty((n, b.obs_dim), dtype=torch.float32, device="cuda:0")
    rew = torch.empty(n, dtype=torch.float32, device="cuda:0")
    te = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    tr = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    resets = 0
    for t in range(steps):
        b.synth_actions(7, t, out=act)
        codes, r0, te0, tr0 = b.step(act)
        assert codes.dtype == torch.uint8 and codes.shape == (n, b.obs_dim)
        b.expand_codes(b.io, 1, obs, rew, te, tr)
        o_obs, o_rew, o_te, o_tr, *_ = ov.step(np_(act))
        assert np.array_equal(np_(obs), o_obs), f"step {t}: obs"
        assert np.array_equal(np_(rew), o_rew.astype(np.float32)), f"step {t}: reward"
        assert np.array_equal(np_(r0), np_(rew)) and np.array_equal(np_(te0), np_(te))
        assert np.array_equal(np_(te).astype(bool), o_te) and np.array_equal(np_(tr).astype(bool), o_tr)
        resets += int((o_te | o_tr).sum())
    assert resets > 0 or steps < 1000
    b.close()


def test_expand_many_blocks_is_one_gather_buffer():
    """W code buffers back to back (a root's [W, io_bytes] gather buffer) expand to the
    W batches' outputs in rank order, reward / terminated / truncated included"""
    cfg = CFG["g20"]
    W, n = 3, 640
    bs = [make(cfg, n, seed=5, env_id_offset=r * n, obs_codes=True) for r in range(W)]
    ref = make(cfg, W * n, seed=5)  # one f32 batch over all W * n global ids
    buf = torch.empty((W, bs[0].io_bytes()), dtype=torch.uint8, device="cuda:0")
    out = (torch.empty((W * n, bs[0].obs_dim), dtype=torch.float32, device="cuda:0"),
           torch.empty(W * n, dtype=torch.float32, device="cuda:0"),
           torch.empty(W * n, dtype=torch.uint8, device="cuda:0"), torch.empty(W * n, dtype=torch.uint8, device="cuda:0"))
    act = torch.empty(W * n, dtype=torch.int32, device="cuda:0")
    for t in range(1005):
        ref.synth_actions(3, t, out=act)
        r_obs, r_rew, r_te, r_tr = ref.step(act)
        for r in range(W):
            bs[r].step(act[r * n:(r + 1) * n].contiguous(), io=buf[r])
        bs[0].expand_codes(buf.view(-1), W, *out)
        if t % 50 == 0 or t >= 995:
            assert torch.equal(out[0], r_obs) and torch.equal(out[1], r_rew), t
            assert torch.equal(out[2], r_te) and torch.equal(out[3], r_tr), t
    for b in bs + [ref]:
        b.close()


def test_expand_codes_rejects_bad_outputs():
    """every caller-supplied output of expand_codes is checked before the raw-pointer
    launch: wrong shape (rows of one block for two), dtype, contiguity or device"""
    cfg = CFG["g20"]
    n = 128
    b = make(cfg, n, obs_codes=True)
    D = b.obs_dim
    src = torch.zeros(2 * b.io_bytes(), dtype=torch.uint8, device="cuda:0")
    f32, u8 = torch.float32, torch.uint8
    good = dict(obs=torch.empty((2 * n, D), dtype=f32, device="cuda:0"),
                reward=torch.empty(2 * n, dtype=f32, device="cuda:0"),
                terminated=torch.empty(2 * n, dtype=u8, device="cuda:0"),
                truncated=torch.empty(2 * n, dtype=u8, device="cuda:0"))
    b.expand_codes(src, 2, **good)  # the right shapes pass
    bad = [("obs", torch.empty((n, D), dtype=f32, device="cuda:0")),
           ("obs", torch.empty((2 * n, D + 1), dtype=f32, device="cuda:0")[:, :D]),
           ("obs", torch.empty((2 * n, D), dtype=f32)),
           ("reward", torch.empty(2 * n, dtype=torch.float64, device="cuda:0")),
           ("terminated", torch.empty(2 * n, dtype=f32, device="cuda:0")),
           ("truncated", torch.empty(n, dtype=u8, device="cuda:0"))]
    for name, t in bad:
        kw = dict(good)
        kw[name] = t
        with pytest.raises(ValueError):
            b.expand_codes(src, 2, **kw)
    b.close()


def test_sharded_codes_one_gpu_no_process_group():
    """ShardedPlantOS(codes=True) without torch.distributed: step_gather / gathered /
    unpack on one GPU equal the f32 batch of the same ids"""
    import torch.distributed as dist
    from plantos_amd.shard import ShardedPlantOS
    assert not dist.is_initialized()
    G, P, Ob, R, C = CFG["g20"]
    n = 4096
    sh = ShardedPlantOS(n, seed=21, codes=True, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R,
                        lidar_channels=C)
    ref = make(CFG["g20"], n, seed=21)
    assert sh.io_bytes() < ref.io_bytes() / 3
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    prev = None
    for t in range(1003):
        ref.synth_actions(4, t, out=act)
        k = sh.step_gather(act)
        r = ref.step(act)
        g = sh.unpack(sh.gathered(k))
        assert all(torch.equal(x, y) for x, y in zip(g, r)), t
        prev = k
    sh.flush()
    assert prev is not None
    sh.close()
    ref.close()
