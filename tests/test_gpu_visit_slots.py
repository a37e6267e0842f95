"""The two visit slots per env (pe_device.hpp vis_env: episode k's visit rows live in
slot k & 1; the prefetch kernel writes the next episode's fresh rows into the idle
slot, so an auto-reset that takes a prefetched record stores no visit row).  The
visits must follow the episode counter through every path that changes it without
a reset: pe_seed(reset_episode_counters) and pe_set_state of the scalars alone --
state and later steps checked against the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu

CFG = (20, 10, 12, 6, 16)


def np_(t):
    return t.detach().cpu().numpy()


def _desync_batch(n, seed, steps):
    """a batch and its oracle, desynchronized and stepped until many envs have reset
    once or twice (odd and even episode counters mixed)"""
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = CFG
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C, seed=seed,
                     device="cuda:0", max_steps=60)
    ov = OracleVec(CFG, np.arange(n), seed, max_steps=60)
    start = (59 - np.random.default_rng(2).integers(0, 60, n)).astype(np.int32)
    sc = np_(b.get_state()["scalars"])
    sc[:, O.S_STEP] = start
    b.set_state(scalars=sc)
    ov.b.scal[:, O.S_STEP] = start
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        o = ov.step(np_(act))
        assert np.array_equal(np_(obs), o[0]), t
    return b, ov, act


def _run_more(b, ov, act, seed, t0, steps):
    for t in range(t0, t0 + steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        o = ov.step(np_(act))
        assert np.array_equal(np_(obs), o[0]), t
        assert np.array_equal(np_(rew), o[1].astype(np.float32)), t
    st = b.get_state()
    assert np.array_equal(np_(st["visits"]), ov.b.visits)
    assert np.array_equal(np_(st["scalars"]), ov.b.scal)


def test_seed_reset_counters_moves_visits():
    seed, n = 41, 1000
    b, ov, act = _desync_batch(n, seed, 130)
    st0 = b.get_state()
    ep = np_(st0["scalars"])[:, O.S_EPISODE]
    assert (ep % 2 == 1).any() and (ep % 2 == 0).any() and (ep >= 2).any()
    b.seed(seed, reset_episode_counters=True)
    st1 = b.get_state()
    assert (np_(st1["scalars"])[:, O.S_EPISODE] == 0).all()
    assert np.array_equal(np_(st1["visits"]), np_(st0["visits"]))
    ov.b.scal[:, O.S_EPISODE] = 0  # the oracle's counters follow (same seed: same later maps)
    _run_more(b, ov, act, seed, 130, 140)
    b.close()


def test_set_state_episode_parity_moves_visits():
    seed, n = 43, 700
    b, ov, act = _desync_batch(n, seed, 90)
    st0 = b.get_state()
    sc = np_(st0["scalars"]).copy()
    sc[:, O.S_EPISODE] += 1 + np.arange(n) % 2  # half the envs change parity
    b.set_state(scalars=sc)
    st1 = b.get_state()
    assert np.array_equal(np_(st1["visits"]), np_(st0["visits"]))
    assert np.array_equal(np_(st1["scalars"])[:, O.S_EPISODE], sc[:, O.S_EPISODE])
    ov.b.scal[:, O.S_EPISODE] = sc[:, O.S_EPISODE]
    _run_more(b, ov, act, seed, 90, 120)
    b.close()


def test_set_state_counter_moved_back_drops_records():
    """episode counters set back by one or two: an env's prefetched record of a later
    episode would become a future key over visit rows since reused -- it must be
    dropped (the reset then generates in place), not taken"""
    seed, n = 47, 700
    b, ov, act = _desync_batch(n, seed, 130)
    st0 = b.get_state()
    sc = np_(st0["scalars"]).copy()
    ep = sc[:, O.S_EPISODE]
    assert (ep >= 2).any()
    sc[:, O.S_EPISODE] = np.maximum(ep - 1 - np.arange(n) % 2, 0)
    b.set_state(scalars=sc)
    st1 = b.get_state()
    assert np.array_equal(np_(st1["visits"]), np_(st0["visits"]))
    ov.b.scal[:, O.S_EPISODE] = sc[:, O.S_EPISODE]
    _run_more(b, ov, act, seed, 130, 140)
    b.close()
