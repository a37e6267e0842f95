"""BASELINE config 5 on one GPU: 524288 envs (20x20, 16 rays, R=6) as the 8 shards
an 8-GPU job runs (rank r: PlantOSBatch(65536, env_id_offset=r*65536), the device-rng
map stream keyed by the GLOBAL env id), stepped 1010 steps across the synchronized
1000-step truncation (the drop-in at A2C_training.py:216-218).

Checks, every step: the 8 shards equal ONE 524288-env handle bit for bit (obs,
reward, terminated, truncated, terminal obs, episode return/length); the oracle
replays sampled global ids of every shard, including ids >= 458752 (the last
shard); and size-independent invariants over all 524288 envs at sampled steps."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu

CFG = (20, 10, 12, 6, 16)
N_SHARD, WORLD = 65536, 8


def _make(n, off, seed):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = CFG
    return PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                        seed=seed, env_id_offset=off, device="cuda:0")


def test_config5_shards_equal_one_batch_and_oracle():
    seed, steps = 21, 1010
    G, C, R = CFG[0], CFG[4], CFG[3]
    n = N_SHARD * WORLD
    big = _make(n, 0, seed)
    shards = [_make(N_SHARD, r * N_SHARD, seed) for r in range(WORLD)]
    # 16 ids per shard: its first, its middle and its last ones
    sample = np.concatenate([r * N_SHARD + np.r_[0:4, 30000:30004, 65000:65004, 65532:65536]
                             for r in range(WORLD)])
    assert sample.max() == n - 1 and (sample >= 458752).sum() == 16
    ov = OracleVec(CFG, sample, seed)
    sidx = torch.as_tensor(sample, device="cuda:0")
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    part = torch.empty(N_SHARD, dtype=torch.int32, device="cuda:0")
    dist = torch.as_tensor(np.float32(np.arange(1, R + 1) / R), device="cuda:0")
    posv = torch.as_tensor(np.float32(np.arange(G) / G), device="cuda:0")
    visv = torch.as_tensor(np.float32(np.arange(11) / 10.0), device="cuda:0")
    for t in range(steps):
        big.synth_actions(seed, t, out=act)
        obs, rew, te, tr = big.step(act)
        for r, sh in enumerate(shards):
            sh.synth_actions(seed, t, out=part)  # keyed by the shard's global ids
            lo, hi = r * N_SHARD, (r + 1) * N_SHARD
            assert torch.equal(part, act[lo:hi]), (t, r)
            o, w, e_, u = sh.step(part)
            assert torch.equal(o, obs[lo:hi]) and torch.equal(w, rew[lo:hi]), (t, r)
            assert torch.equal(e_, te[lo:hi]) and torch.equal(u, tr[lo:hi]), (t, r)
            if t >= 999:  # the truncation step and after: terminal outputs of the shard
                assert torch.equal(sh.terminal_obs, big.terminal_obs[lo:hi]), (t, r)
                assert torch.equal(sh.episode_return, big.episode_return[lo:hi]), (t, r)
                assert torch.equal(sh.episode_length, big.episode_length[lo:hi]), (t, r)
        o_obs, o_rew, o_te, o_tr, o_tobs, o_ret, o_len = ov.step(act[sidx].cpu().numpy())
        assert (obs[sidx].cpu().numpy() == o_obs).all(), t
        assert (rew[sidx].cpu().numpy() == o_rew.astype(np.float32)).all(), t
        assert (te[sidx].cpu().numpy().astype(bool) == o_te).all(), t
        assert (tr[sidx].cpu().numpy().astype(bool) == o_tr).all(), t
        done = o_te | o_tr
        if done.any():
            assert (big.terminal_obs[sidx].cpu().numpy()[done] == o_tobs[done]).all(), t
            assert (big.episode_return[sidx].cpu().numpy()[done] == o_ret[done]).all(), t
            assert (big.episode_length[sidx].cpu().numpy()[done] == o_len[done]).all(), t
        if t in (0, 500, 998, 999, 1000, steps - 1):
            lid = obs[:, :5 * C].reshape(n, C, 5)
            assert bool((lid[:, :, 1:].sum(-1) == 1.0).all()), t
            assert bool(torch.isin(lid[:, :, 0], dist).all()), t
            assert bool(torch.isin(obs[:, 5 * C:5 * C + 2], posv).all()), t
            assert bool(torch.isin(obs[:, 5 * C + 2:], visv).all()), t
            assert int(tr.sum()) == (n if t == 999 else 0), t  # synchronized episodes
    s = big.get_state(parts=("scalars",))["scalars"].cpu().numpy()
    assert (s[sample] == ov.b.scal).all()
    assert (s[:, O.S_EPISODE] == 1 + steps // 1000).all() and (s[:, O.S_STEP] == steps % 1000).all()
    for r, sh in enumerate(shards):
        ss = sh.get_state(parts=("scalars",))["scalars"]
        assert torch.equal(ss.cpu(), torch.as_tensor(s[r * N_SHARD:(r + 1) * N_SHARD])), r
        sh.close()
    big.close()
