"""GPU parity of the step kernel's auto-reset paths against the oracle with
DESYNCHRONIZED episodes (every env starts at its own step count, so a few envs
reset in every step, as in steady-state training): prefetched resets (maps
generated ahead by pe_prefetch_kernel, at several launch cadences, across a seed
change), the wave-cooperative reset (pe_coop.hpp) and, forced through
pe_config.coop_max_done / prefetch_every, every path for dense resets.  Every output of every step is
compared, plus the terminal info rows and the final state.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu

CFG = {
    "g20": (20, 10, 12, 6, 16),
    "g64": (64, 100, 120, 6, 64),
    "g7": (7, 3, 3, 3, 12),        # runtime sector kernel, one-word
    "g32": (32, 20, 30, 9, 24),    # runtime sector kernel, multi-word
    "g21": (21, 8, 50, 2, 10),
    "g25": (25, 10, 12, 6, 16),   # the multi-word C16 sector kernel (train_mcts's grid)
    "g15": (15, 6, 8, 4, 16),     # one-word C16R4 sector kernel (test_environment.py:24)
    "g12r2": (12, 4, 6, 2, 10),   # one-word C10R2
    "g64r32": (64, 100, 120, 32, 64),  # the far sector kernel (long rays, pe_step_far)
    "g30r2": (30, 12, 40, 2, 10),  # multi-word C10R2
    "g16c40": (16, 6, 8, 5, 40),   # C > 32: the runtime sector kernel, byte-coded tile
    "g40c48": (40, 100, 120, 8, 48),  # the same, multi-word rows (bench geometry)
}


def np_(t):
    return t.detach().cpu().numpy()


def info_rows(b, idx):
    rows = np.zeros((len(idx), 11), np.int32)
    for k, e in enumerate(idx):
        th, hy, tot, ex, tc = b.info(e)
        s = b.scal[e]
        rows[k] = [s[O.S_X], s[O.S_Y], th, hy, tot, s[O.S_STEP], ex, tc, s[O.S_COLLIDED], s[O.S_COLL], s[O.S_POISONED]]
    return rows


@pytest.mark.parametrize("name,n,steps,spread,coop_max,every,reseed_at,reset_at,side", [
    ("g20", 2048, 160, 150, None, None, None, None, False),   # sparse: prefetched / cooperative resets
    ("g64", 192, 50, 40, None, None, None, None, False),      # 64x64: cooperative resets always
    ("g7", 700, 120, 100, None, None, None, None, False),
    ("g32", 300, 60, 50, None, None, None, None, False),
    ("g21", 400, 60, 50, None, None, None, None, False),
    ("g25", 600, 80, 60, None, None, None, None, False),
    ("g15", 600, 80, 60, None, None, None, None, False),
    ("g12r2", 600, 80, 60, None, None, None, None, False),
    ("g30r2", 400, 60, 50, None, None, None, None, False),
    ("g16c40", 300, 60, 50, None, None, None, None, False),
    ("g40c48", 256, 60, 50, None, None, None, None, False),
    ("g40c48", 128, 12, 1, "64", None, None, None, False),    # every env at once, cooperative, byte-coded records
    ("g64r32", 192, 50, 40, None, None, None, None, False),
    ("g64r32", 128, 12, 1, "0", None, None, None, False),    # dense: serial resets (coop_max_done 0)
    ("g21", 256, 12, 1, "0", None, None, None, False),        # the constructor default, dense: lane-per-env path
    ("g20", 256, 12, 1, "64", None, None, None, False),       # every env at once through the cooperative path
    ("g64", 128, 12, 1, "0", None, None, None, False),        # every env at once through the lane-per-env path
    ("g20", 256, 12, 1, "8", "0", None, None, False),         # no prefetch: in-kernel map generation
    ("g20", 1024, 80, 60, None, "1", None, None, False),      # prefetch launch after every step
    ("g20", 1024, 80, 60, None, "7", None, None, False),
    ("g32", 300, 60, 50, None, "0", None, None, False),
    ("g20", 1024, 80, 60, None, "5", 30, None, False),        # new seed mid-run: prefetched maps dropped
    ("g64", 192, 40, 30, None, "3", 15, None, False),
    ("g20", 1024, 80, 60, None, "16", None, 33, False),  # reset() of every env mid-run (prefetch refill)
    ("g64", 192, 40, 30, None, None, None, 17, False),
    ("g20", 1024, 80, 60, None, "1", 30, None, True),  # steps + reseed on a side stream
])
def test_desync_autoreset_parity(name, n, steps, spread, coop_max, every, reseed_at, reset_at, side):
    """coop_max / every: pe_config.coop_max_done / prefetch_every (steps between
    prefetch launches; "0" = off).  side: everything on a non-default torch stream
    (pe_seed must clear the prefetched records on THAT stream, after the queued
    prefetch launches)."""
    import contextlib
    ctx = torch.cuda.stream(torch.cuda.Stream()) if side else contextlib.nullcontext()
    with ctx:
        _desync_run(name, n, steps, spread, coop_max, every, reseed_at, reset_at)


@pytest.mark.parametrize("name,n,steps,spread,coop_max", [
    ("g20", 2048, 160, 150, None),  # one-done blocks: the early record (4-code words) + the info wave
    ("g20", 1024, 80, 60, "64"),    # several done envs per block, cooperative, code records
    ("g20", 256, 12, 1, None),      # every env at once: lane-per-env resets, fresh codes from HBM
    ("g64", 192, 50, 40, None),     # 64x64: the LDS-DMA staged record
])
def test_desync_autoreset_parity_codes(name, n, steps, spread, coop_max):
    """The byte-coded step (pe_step_codes, config 5's codes gather) through the same
    desynchronized auto-reset paths: expanded obs, terminal obs / info / return /
    length and the final state equal the oracle's."""
    _desync_run(name, n, steps, spread, coop_max, None, None, None, codes=True)


def _desync_run(name, n, steps, spread, coop_max, every, reseed_at, reset_at, codes=False):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = cfg = CFG[name]
    seed = aseed = 31
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C, seed=seed,
                     device="cuda:0", coop_max_done=None if coop_max is None else int(coop_max),
                     prefetch_every=None if every is None else int(every), obs_codes=codes)
    f_obs = torch.empty((n, b.obs_dim), dtype=torch.float32, device="cuda:0") if codes else None
    ov = OracleVec(cfg, np.arange(n), seed)
    # desynchronize: env e starts at step 1000 - 1 - k(e), k in [0, spread)
    rng = np.random.default_rng(5)
    start = (999 - rng.integers(0, spread, n)).astype(np.int32)
    sc = np_(b.get_state()["scalars"])
    sc[:, O.S_STEP] = start
    b.set_state(scalars=sc)
    ov.b.scal[:, O.S_STEP] = start
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    resets = 0
    for t in range(steps):
        if t == reseed_at:  # map stream of every later reset keyed by the new seed
            seed = 977
            b.seed(seed, reset_episode_counters=False)
        if t == reset_at:  # reset() of every env: new maps, then the next ones prefetched again
            r_obs = np_(b.reset()).copy()
            for k in range(n):
                ov.b.reset_philox(k, seed, k, int(ov.b.scal[k, O.S_EPISODE]))
                ov.ret[k] = 0.0
            assert (r_obs == ov.b.obs()).all()
            # desynchronize again, so that the refilled records are consumed in the window
            st2 = (999 - rng.integers(0, steps - t - 3, n)).astype(np.int32)
            sc = np_(b.get_state()["scalars"])
            sc[:, O.S_STEP] = st2
            b.set_state(scalars=sc)
            ov.b.scal[:, O.S_STEP] = st2
        b.synth_actions(aseed, t, out=act)
        a_np = np_(act)
        obs, rew, te, tr = b.step(act)
        if codes:  # the step wrote byte codes: expand them (pe_expand_obs_codes)
            obs = b.expand_codes(b.io, 1, f_obs)[0]
        # oracle: step, pre-reset info of the done envs, then the resets (OracleVec.step)
        o_obs, o_rew, o_te, o_tr = ov.b.step(a_np)
        done = o_te | o_tr
        didx = np.nonzero(done)[0]
        o_info = info_rows(ov.b, didx)
        o_tobs = o_obs.copy()
        ov.ret += o_rew
        o_ret, o_len = ov.ret.copy(), ov.b.scal[:, O.S_STEP].copy()
        for k in didx:
            ov.b.reset_philox(int(k), seed, int(k), int(ov.b.scal[k, O.S_EPISODE]))
            ov.ret[k] = 0.0
        if len(didx):
            o_obs[done] = ov.b.obs(didx)[done]
        resets += len(didx)
        assert (np_(rew) == o_rew.astype(np.float32)).all(), t
        assert (np_(te).astype(bool) == o_te).all() and (np_(tr).astype(bool) == o_tr).all(), t
        assert (np_(obs) == o_obs).all(), t
        if len(didx):
            assert (np_(b.terminal_obs)[didx] == o_tobs[didx]).all(), t
            assert (np_(b.episode_return)[didx] == o_ret[didx]).all(), t
            assert (np_(b.episode_length)[didx] == o_len[didx]).all(), t
            assert (np_(b.terminal_info)[didx] == o_info).all(), t
    assert resets >= n  # every env reset at least once
    st = b.get_state()
    assert (np_(st["cells"]) == ov.b.cells).all()
    assert (np_(st["visits"]) == ov.b.visits).all()
    assert (np_(st["scalars"]) == ov.b.scal).all()
    b.close()


def test_desync_curriculum_cooperative_reset():
    """CurriculumWrapper (visit counts carried into the next episode, explored map
    restarted) through the cooperative reset: state after sparse resets equals the
    lane-per-env path's (coop_max_done=0) on the same inputs."""
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = CFG["g20"]
    n, steps = 512, 60
    outs = []
    for cm in (8, 0):
        b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                         seed=3, device="cuda:0", coop_max_done=cm)
        b.enable_curriculum(initial_threshold=5.0, max_threshold=100.0)
        sc = np_(b.get_state()["scalars"])
        sc[:, O.S_STEP] = 999 - np.random.default_rng(2).integers(0, 50, n)
        b.set_state(scalars=sc)
        act = torch.empty(n, dtype=torch.int32, device="cuda:0")
        trace = []
        for t in range(steps):
            b.synth_actions(3, t, out=act)
            obs, rew, te, tr = b.step(act)
            trace.append((np_(obs).copy(), np_(rew).copy(), np_(te).copy(), np_(tr).copy()))
        st = {k: np_(v).copy() for k, v in b.get_state().items()}
        outs.append((trace, st, [np_(x).copy() for x in b.get_curriculum()]))
        b.close()
    (ta, sa, ca), (tb, sb, cb) = outs
    for x, y in zip(ta, tb):
        for u, v in zip(x, y):
            assert (u == v).all()
    for k in sa:
        assert (sa[k] == sb[k]).all(), k
    for u, v in zip(ca, cb):
        assert (u == v).all()
