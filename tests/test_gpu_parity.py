"""GPU parity: the HIP hot path (through the C-ABI) vs the oracle / reference fixtures.

Bar: bit-exact integer state and obs; reward bit-exact to float32(reference f64)
(tolerance 0 -- stricter than north_star's 1e-6); episode returns bit-exact f64.
"""
import numpy as np
import pytest
import torch

from golden_util import INJECT_CFGS, TRAJ_FILES, cfg_tuple, load
from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu

CFG = {
    "g20": (20, 10, 12, 6, 16),
    "g21": (21, 8, 50, 2, 10),
    "g25": (25, 10, 12, 6, 16),
    "g64": (64, 100, 120, 6, 64),
    "g64r32": (64, 100, 120, 32, 64),
    "g7": (7, 3, 3, 3, 12),
    "g32": (32, 20, 30, 9, 24),
    "g15": (15, 6, 8, 4, 16),     # test_environment.py:24's custom env (one-word C16R4 sector kernel)
    "g25r4": (25, 10, 12, 4, 16),  # multi-word C16R4
    "g12r2": (12, 4, 6, 2, 10),    # one-word C10R2 (g21 = the constructor default: multi-word C10R2)
    "g30r2": (30, 12, 40, 2, 10),  # multi-word C10R2 (G + 2R > 32)
    "g8r12": (8, 3, 3, 12, 16),    # R > G: runtime sector kernel, window rows mostly off the map
    "g8r20": (8, 3, 3, 20, 16),    # R > 14 and > G: the wave kernel's raw-window ray path (no rover-aligned re-staging)
    "g16c40": (16, 6, 8, 5, 40),   # C > 32: the runtime sector kernel with the byte-coded tile
    "g24c100": (24, 10, 12, 8, 100),  # C = 100 (near the 120-ray LDS bound): wave kernel, rays past lane 63
}

# which step kernel each geometry runs (pe_kernel_name): the sector kernel wherever a
# specialization exists, the table-driven kernel otherwise
KERNELS = {
    "g20": "pe_step_quad<C16,R6,1word>", "g25": "pe_step_quad<C16,R6>", "g64": "pe_step_quad<C64,R6,bytetile>",
    "g21": "pe_step_quad<C10,R2>", "g12r2": "pe_step_quad<C10,R2,1word>", "g30r2": "pe_step_quad<C10,R2>", "g15": "pe_step_quad<C16,R4,1word>",
    "g25r4": "pe_step_quad<C16,R4>", "g64r32": "pe_step_far<C64,R32,bytetile>", "g7": "pe_step_quad<runtime C,R,1word>",
    "g32": "pe_step_quad<runtime C,R>", "g8r12": "pe_step_quad<runtime C,R,1word>", "g24c100": "pe_step_wave",
    "g8r20": "pe_step_wave", "g16c40": "pe_step_quad<runtime C,R,1word,bytetile>",
}


def make(cfg, n, **kw):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = cfg
    return PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                        device="cuda:0", **kw)


def np_(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name", INJECT_CFGS)
def test_injected_step_parity(name):
    f = load(f"inject_{name}")
    cfg = cfg_tuple(f)
    n = f["cells"].shape[0]
    b = make(cfg, n, autoreset=False)
    scal = np.zeros((n, 8), np.int32)
    scal[:, :6] = f["scal"]
    b.set_state(cells=f["cells"], visits=f["visits"].astype(np.int32), explored=f["explored"], scalars=scal)
    obs_pre = np_(b.reset(mask=np.zeros(n, np.uint8)))
    assert (obs_pre == f["obs_pre"]).all()
    obs, rew, te, tr = b.step(torch.as_tensor(f["action"], dtype=torch.int32, device="cuda:0"))
    assert (np_(obs) == f["obs"]).all()
    assert (np_(rew) == f["reward"].astype(np.float32)).all()
    assert (np_(te).astype(bool) == f["term"].astype(bool)).all()
    assert (np_(tr).astype(bool) == f["trunc"].astype(bool)).all()
    st = b.get_state()
    assert (np_(st["cells"]) == f["cells_post"]).all()
    assert (np_(st["visits"]) == f["visits_post"].astype(np.int32)).all()
    assert (np_(st["explored"]) == f["explored_post"]).all()
    sp = f["scal_post"]
    s = np_(st["scalars"])
    assert (s[:, :6] == sp[:, :6]).all()
    assert ((s[:, 6] & 1).astype(bool) == f["root_raises"].astype(bool)).all()
    info = np_(b.get_info())
    from plantos_amd import _capi as C
    assert (info[:, C.PE_I_EXPLORED] == sp[:, 6]).all()
    assert (info[:, C.PE_I_TOTAL_CELLS] == sp[:, 7]).all()
    assert (info[:, C.PE_I_THIRSTY] == sp[:, 8]).all()
    assert (info[:, C.PE_I_HYDRATED] == sp[:, 9]).all()
    b.close()


def test_kat_seed0_gpu():
    """Appendix B through the GPU: reference map loaded, 1000 reference actions."""
    k = load("kat_seed0")
    b = make(cfg_tuple(k), 1)
    obs0 = np_(b.load_maps([0], k["cells0"][None], k["rover0"][None]))
    assert (obs0[0] == k["obs"][0]).all()
    acts = torch.as_tensor(k["actions"], dtype=torch.int64, device="cuda:0")
    for t in range(1000):
        obs, rew, te, tr = b.step(acts[t:t + 1])
        assert float(np_(rew)[0]) == np.float32(k["reward"][t]), t
        assert bool(np_(te)[0]) == bool(k["terminated"][t]) and bool(np_(tr)[0]) == bool(k["truncated"][t]), t
        if t < 999:
            assert (np_(obs)[0] == k["obs"][t + 1]).all(), t
    # step 1000 truncates: terminal obs is the reference's final obs, return is the f64 sum
    assert (np_(b.terminal_obs)[0] == k["obs"][1000]).all()
    assert float(np_(b.episode_return)[0]) == float(k["reward_sum"])
    assert int(np_(b.episode_length)[0]) == 1000
    b.close()


@pytest.mark.parametrize("name", TRAJ_FILES)
def test_dummyvecenv_trajectory_gpu(name):
    """Reference DummyVecEnv rollouts; reset layouts supplied from the fixture
    (CPython-stream mode), everything else computed on the GPU."""
    f = load(name)
    acts = f["actions"]
    T, N = acts.shape
    b = make(cfg_tuple(f), N)
    obs0 = np_(b.load_maps(np.arange(N), f["maps0"], f["rover0"]))
    assert (obs0 == f["obs0"]).all()
    ri = 0
    for t in range(T):
        obs, rew, te, tr = b.step(torch.as_tensor(acts[t], device="cuda:0"))
        obs = np_(obs).copy()
        assert (np_(rew) == f["reward"][t].astype(np.float32)).all(), t
        te_, tr_ = np_(te).astype(bool), np_(tr).astype(bool)
        assert (te_ == f["terminated"][t].astype(bool)).all() and (tr_ == f["truncated"][t].astype(bool)).all()
        done = np.nonzero(te_ | tr_)[0]
        if len(done):
            tobs = np_(b.terminal_obs)
            for e in done:
                assert (tobs[e] == f["terminal_obs"][t, e]).all()
            sel = np.arange(ri, ri + len(done))
            assert (f["reset_t"][sel] == t).all() and (f["reset_env"][sel] == done).all()
            fresh = np_(b.load_maps(done, f["reset_cells"][sel], f["reset_rover"][sel]))
            obs[done] = fresh
            ri += len(done)
        assert (obs == f["obs"][t]).all(), t
    b.close()


@pytest.mark.parametrize("name", ["g20", "g21", "g64", "g7", "g32", "g64r32"])
def test_device_reset_matches_oracle_philox(name):
    cfg = CFG[name]
    n = 512 if cfg[0] <= 32 else 128
    b = make(cfg, n, seed=1234)
    st = {k: np_(v) for k, v in b.get_state().items()}
    ob = O.Batch(O.config(*cfg), n)
    for e in range(n):
        ob.reset_philox(e, 1234, e, 0)
    assert (st["cells"] == ob.cells).all()
    assert (st["visits"] == ob.visits).all()
    assert (st["explored"] == ob.explored).all()
    assert (st["scalars"] == ob.scal).all()
    assert (np_(b.reset(mask=np.zeros(n, np.uint8))) == ob.obs()).all()
    b.close()


@pytest.mark.parametrize("name", sorted(KERNELS))
def test_kernel_selection(name):
    b = make(CFG[name], 64)
    # the headline geometry's small batches run 16-env workgroups (see below)
    assert b.kernel_name == (KERNELS[name][:-1] + ",W8,E16>" if name == "g20" else KERNELS[name])
    b.close()


# the headline geometry above 32768 envs: the 64-env sector kernel (the persistent
# pipelined one, pe_pipe.hpp, measured slower: a debug-build A/B only)
BIG_KERNEL = "pe_step_quad<C16,R6,1word>"


@pytest.mark.parametrize("n,suffix", [(1, ",W8,E16"), (4096, ",W8,E16"), (4097, ",E16"), (8192, ",E16"),
                                      (8193, ",E32"), (32768, ",E32"), (32769, None), (65536, None)])
def test_small_batch_workgroup_shape(n, suffix):
    """Batches too small for four 64-env workgroups per CU run 16- or 32-env
    workgroups of the same kernel, up to 4096 envs with 8 waves (sectors of 2 rays);
    larger ones 64-env workgroups -- pe_create's choice, by batch size"""
    b = make(CFG["g20"], n)
    assert b.kernel_name == (BIG_KERNEL if suffix is None else "pe_step_quad<C16,R6,1word" + suffix + ">")
    b.close()


@pytest.mark.parametrize("name,n,steps", [("g20", 4096, 1100), ("g21", 1000, 1010), ("g7", 777, 400),
                                          ("g64", 256, 120), ("g64r32", 96, 60), ("g25", 300, 200),
                                          ("g15", 1000, 1010), ("g25r4", 300, 200), ("g12r2", 500, 300),
                                          ("g32", 400, 300), ("g8r12", 300, 300), ("g24c100", 200, 120),
                                          ("g30r2", 300, 200), ("g8r20", 300, 200), ("g16c40", 300, 200)])
def test_rollout_parity_device_rng(name, n, steps):
    """Device-rng episodes with synthetic actions, auto-reset included (g20 crosses
    the 1000-step truncation): every output of every step vs the oracle."""
    cfg = CFG[name]
    seed = 77
    b = make(cfg, n, seed=seed)
    ov = OracleVec(cfg, np.arange(n), seed)
    assert (np_(b.reset(mask=np.zeros(n, np.uint8))) == ov.obs()).all()
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        a_np = np_(act)
        if t == 0:
            assert all(a_np[e] == O.synth_action(seed, e, 0) for e in range(0, n, max(1, n // 50)))
        obs, rew, te, tr = b.step(act)
        o_obs, o_rew, o_te, o_tr, o_tobs, o_ret, o_len = ov.step(a_np)
        assert (np_(rew) == o_rew.astype(np.float32)).all(), t
        assert (np_(te).astype(bool) == o_te).all() and (np_(tr).astype(bool) == o_tr).all(), t
        assert (np_(obs) == o_obs).all(), t
        done = o_te | o_tr
        if done.any():
            assert (np_(b.terminal_obs)[done] == o_tobs[done]).all()
            assert (np_(b.episode_return)[done] == o_ret[done]).all()
            assert (np_(b.episode_length)[done] == o_len[done]).all()
    st = b.get_state()
    assert (np_(st["visits"]) == ov.b.visits).all()
    assert (np_(st["cells"]) == ov.b.cells).all()
    assert (np_(st["scalars"]) == ov.b.scal).all()
    b.close()


@pytest.mark.parametrize("name,desync,n", [("g20", False, 65536), ("g20", True, 65536), ("g64", False, 65536),
                                           ("g64", True, 65536), ("g64r32", True, 65536), ("g25", False, 65536),
                                           ("g25", True, 65536),
                                           # the runtime kernel switched to the byte tile at full batch (C = 24)
                                           ("g32", True, 65536),
                                           # BASELINE config 2 (16-env workgroups) and a 32-env-workgroup batch
                                           ("g20", False, 4096), ("g20", True, 4096), ("g20", True, 20000),
                                           # a ragged last block
                                           ("g20", True, 40001)])
def test_full_batch_sampled_parity_and_invariants(name, desync, n):
    """65536 envs (BASELINE headline 20x20/16 rays, the 64x64/64-ray stress config,
    and 25x25/16 rays -- the geometry the reference's training scripts build,
    A2C_training.py:206-212, trainingCode.py:121-125) for 1010+ steps, crossing the 1000-step truncation: the oracle replays
    192 sampled global env ids (envs are independent) every step, and size-
    independent invariants hold over ALL envs (one-hot per ray, distances in {r/R},
    positions in {x/G}, slice values in {k/10}, episode counts and step counts
    after the truncations).  desync: every env starts at its own step count in
    [0, 1000) -- ~65 auto-resets in every step through the prefetched /
    cooperative reset paths."""
    cfg = CFG[name]
    G, C, R = cfg[0], cfg[4], cfg[3]
    seed, steps = 5, 1010 if name.startswith("g64") else 1100
    b = make(cfg, n, seed=seed)
    sample = np.unique(np.r_[0:64, n // 2 - 32:n // 2 + 32, n - 64:n])
    ov = OracleVec(cfg, sample, seed)
    start = np.zeros(n, np.int32)
    if desync:
        start = np.random.default_rng(11).integers(0, 1000, n).astype(np.int32)
        sc = np_(b.get_state(parts=("scalars",))["scalars"])
        sc[:, O.S_STEP] = start
        b.set_state(scalars=sc)
        ov.b.scal[:, O.S_STEP] = start[sample]
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    sidx = torch.as_tensor(sample, device="cuda:0")
    dist = np.float32(np.arange(1, R + 1) / R)
    posv = np.float32(np.arange(G) / G)
    visv = np.float32(np.arange(11) / 10.0)
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        o_obs, o_rew, o_te, o_tr, o_tobs, o_ret, o_len = ov.step(np_(act[sidx]))
        assert (np_(rew[sidx]) == o_rew.astype(np.float32)).all(), t
        assert (np_(te[sidx]).astype(bool) == o_te).all() and (np_(tr[sidx]).astype(bool) == o_tr).all(), t
        done = o_te | o_tr
        if done.any():
            assert (np_(b.terminal_obs[sidx])[done] == o_tobs[done]).all(), t
            assert (np_(b.episode_return[sidx])[done] == o_ret[done]).all(), t
            assert (np_(b.episode_length[sidx])[done] == o_len[done]).all(), t
        if not (t % 50 == 0 or t in (999, 1000)) and done.any():
            assert (np_(obs[sidx]) == o_obs).all(), t  # fresh reset obs of the sampled done envs
        if t % 50 == 0 or t in (999, 1000):
            ob = np_(obs)
            assert (ob[sample] == o_obs).all(), t
            lid = ob[:, :5 * C].reshape(n, C, 5)
            assert (lid[:, :, 1:].sum(-1) == 1.0).all(), t
            assert np.isin(lid[:, :, 0], dist).all(), t
            assert np.isin(ob[:, 5 * C:5 * C + 2], posv).all(), t
            assert np.isin(ob[:, 5 * C + 2:], visv).all(), t
    st = b.get_state(parts=("scalars", "visits"))
    s = np_(st["scalars"])
    assert (s[sample] == ov.b.scal).all()
    # exact visit counts, past 15 too: the headline kernel defers its overflow writes to the
    # next step (pe_device.hpp vx_pending), get_state applies the pending ones first
    vis = np_(st["visits"][torch.as_tensor(sample, device=st["visits"].device)])
    assert (vis == ov.b.visits.reshape(vis.shape)).all()
    if desync and G <= 25:  # episodes of up to ~1000 steps at the end: the overflow path ran
        assert (vis >= 15).any()
    # a random policy never finishes a map: every episode ends at the truncation
    assert (s[:, O.S_EPISODE] == 1 + (start + steps) // 1000).all()
    assert (s[:, O.S_STEP] == (start + steps) % 1000).all()
    b.close()


def test_determinism_and_sharding_equivalence():
    """Same seed => identical outputs; two shards with env_id_offset reproduce one big batch."""
    cfg = CFG["g20"]
    n = 4096
    full = make(cfg, n, seed=9)
    lo = make(cfg, n // 2, seed=9, env_id_offset=0)
    hi = make(cfg, n // 2, seed=9, env_id_offset=n // 2)
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(1005):
        full.synth_actions(3, t, out=act)
        o, r, _, _ = full.step(act)
        o1, r1, _, _ = lo.step(act[: n // 2].clone())
        o2, r2, _, _ = hi.step(act[n // 2:].clone())
        if t % 100 == 0 or t > 995:
            assert torch.equal(o[: n // 2], o1) and torch.equal(o[n // 2:], o2)
            assert torch.equal(r[: n // 2], r1) and torch.equal(r[n // 2:], r2)
    for x in (full, lo, hi):
        x.close()


@pytest.mark.parametrize("name,n", [(nm, k) for nm in ("g20", "g16c40", "g8r20") for k in (1, 63, 65, 1000)] +
                         [("g64r32", k) for k in (1, 63, 65)])
def test_ragged_batch_sizes(n, name):
    """int64 actions (8-byte action words) and partial workgroups, through the sector
    kernel, both ray paths of the one-wave-per-env kernel and the far kernel (g64r32:
    its off-map quadrant rows are loaded unclamped, so a one-env batch reads the slack
    pe_create keeps around the grid array on both sides)"""
    cfg = CFG[name]
    b = make(cfg, n, seed=3)
    if name == "g64r32":
        assert b.kernel_name == KERNELS[name]
    ov = OracleVec(cfg, np.arange(n), 3)
    for t in range(30):
        a = np.array([O.synth_action(11, e, t) for e in range(n)], np.int64)
        obs, rew, te, tr = b.step(torch.as_tensor(a, device="cuda:0"))  # int64 actions
        o_obs, o_rew, *_ = ov.step(a)
        assert (np_(obs) == o_obs).all() and (np_(rew) == o_rew.astype(np.float32)).all()
    b.close()


@pytest.mark.parametrize("name", ["g20", "g16c40"])
def test_out_of_range_actions(name):
    """Negative actions wrap like Python list indices (plantos_env.py:187); < -4 is the
    reference's IndexError, flagged (bit1); >= 4 waters (plantos_env.py:168-169) -- in
    the sector kernel and the one-wave-per-env kernel (int64 actions)."""
    cfg = CFG[name]
    n = 64
    b = make(cfg, n, seed=4, autoreset=False)
    ov = OracleVec(cfg, np.arange(n), 4)
    rng = np.random.default_rng(0)
    for t in range(50):
        a = rng.integers(-6, 9, n).astype(np.int64)
        obs, rew, te, tr = b.step(torch.as_tensor(a, device="cuda:0"))
        o_obs, o_rew, o_te, o_tr = ov.b.step(a)
        assert (np_(obs) == o_obs).all() and (np_(rew) == o_rew.astype(np.float32)).all()
    assert b.poll_errors() & 2
    s = np_(b.get_state()["scalars"])
    assert (s == ov.b.scal).all()
    b.close()


def test_lds_bounds_of_the_ray_count():
    """lidar_channels beyond the LDS obs tile of the lane-per-env reset / load_maps
    kernels (C > 120) is refused at create, not launched"""
    from plantos_amd import PlantOSBatch
    with pytest.raises(ValueError, match="LDS"):
        PlantOSBatch(8, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=200,
                     device="cuda:0")
    PlantOSBatch(8, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=120,
                 device="cuda:0").close()
    # the bound depends on R too: the ray offsets (2CR bytes) share the 160 KiB
    with pytest.raises(ValueError, match="LDS"):
        PlantOSBatch(8, grid_size=20, num_plants=10, num_obstacles=12, lidar_range=8, lidar_channels=120,
                     device="cuda:0")


def test_no_room_raises():
    from plantos_amd import PlantOSBatch
    # G=5: one obstacle cluster of >= 4 cells leaves <= 21 free cells < 22 + 1
    with pytest.raises(ValueError):
        PlantOSBatch(8, grid_size=5, num_plants=22, num_obstacles=3, lidar_range=2, lidar_channels=4,
                     device="cuda:0")


def test_terminating_explorer_episode():
    """Termination + completion bonus (plantos_env.py:176-181) on the GPU: a map
    with one free cell left, then a move into it."""
    cfg = CFG["g7"]
    f = load("inject_g7")
    idx = np.nonzero(f["term"])[0]
    n = len(idx)
    b = make(cfg, n, autoreset=True, seed=1)
    scal = np.zeros((n, 8), np.int32)
    scal[:, :6] = f["scal"][idx]
    b.set_state(cells=f["cells"][idx], visits=f["visits"][idx].astype(np.int32), explored=f["explored"][idx],
                scalars=scal)
    obs, rew, te, tr = b.step(torch.as_tensor(f["action"][idx], device="cuda:0"))
    assert np_(te).all()
    assert (np_(rew) == f["reward"][idx].astype(np.float32)).all()
    assert (np_(b.terminal_obs) == f["obs"][idx]).all()
    b.close()
