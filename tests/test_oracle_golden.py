"""Pin the CPU oracle (oracle/plantos_oracle.c) against the reference's own outputs.

Every fixture in tests/golden/ was produced by running the reference
(/root/reference/plantos_env.py and gradio-app/plantos_env_new.py) through
tools/gen_golden.py.  These tests make the oracle trustworthy as the checker
for the HIP path (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

from golden_util import INJECT_CFGS, MAP_CFGS, TRAJ_FILES, cfg_tuple, load
from oracle import oracle as O


def test_kat_seed0_appendix_b():
    """random.seed(0); reset; 1000 steps (fork semantics)."""
    k = load("kat_seed0")
    cfg = O.config(*cfg_tuple(k))
    b = O.Batch(cfg, 1)
    b.reset_cpython(0, O.MT(0))
    assert (b.cells[0] == k["cells0"]).all()
    assert tuple(b.scal[0, :2]) == tuple(k["rover0"]) == (12, 19)
    assert (b.obs()[0] == k["obs"][0]).all()
    total = 0.0
    for t, a in enumerate(k["actions"]):
        o, r, te, tr = b.step([a])
        total += r[0]
        assert (o[0] == k["obs"][t + 1]).all(), t
        assert r[0] == k["reward"][t], t
        assert te[0] == k["terminated"][t] and tr[0] == k["truncated"][t], t
        assert tuple(b.scal[0, :2]) == tuple(k["rover"][t])
        assert b.info(0)[3] == k["explored"][t]
        assert b.scal[0, O.S_COLL] == k["collisions"][t]
    assert total == k["reward_sum"] == -670.0000000000028
    assert (b.visits[0] == k["final_visits"]).all()
    assert (b.explored[0] == k["final_explored"]).all()
    assert b.visits[0].sum() == 735


def test_kat_root_env_poison_step():
    """The root env raises TypeError at the first hydrated watering (plantos_env.py:217-220);
    the oracle flags that step (S_POISONED bit 0) instead, with fork reward -10.1."""
    k = load("kat_seed0")
    b = O.Batch(O.config(*cfg_tuple(k)), 1)
    b.reset_cpython(0, O.MT(0))
    s = 0.0
    for t, a in enumerate(k["actions"]):
        before = b.scal[0, O.S_POISONED]
        _, r, _, _ = b.step([a])
        if b.scal[0, O.S_POISONED] & 1 and not before & 1:
            assert t == int(k["root_raise_step"]) == 818
            assert r[0] == -10.1
            break
        s += r[0]
    assert s == k["root_reward_sum"]


@pytest.mark.parametrize("cfg", MAP_CFGS)
def test_cpython_reset_stream(cfg):
    """random.seed(s) then successive reset(): obstacles, plants (incl. thirsty draws),
    rover, and the exact number of MT draws consumed (next getrandbits(32))."""
    f = load(f"maps_{cfg}")
    c = O.config(*cfg_tuple(f))
    seeds = f["seeds"]
    K = f["cells"].shape[1]
    for si, s in enumerate(seeds):
        mt = O.MT(int(s))
        b = O.Batch(c, 1)
        for kk in range(K):
            b.reset_cpython(0, mt)
            assert (b.cells[0] == f["cells"][si, kk]).all(), (s, kk)
            assert tuple(b.scal[0, :2]) == tuple(f["rover"][si, kk]), (s, kk)
            if kk == 0:
                assert (b.obs()[0] == f["obs0"][si]).all()
        assert mt.u32() == f["next_u32"][si]


@pytest.mark.parametrize("cfg", INJECT_CFGS)
def test_injected_steps(cfg):
    """State-injected single steps: obs of the injected state, then step outputs and
    the full post-step state, bit-exact (reward compared as f64)."""
    f = load(f"inject_{cfg}")
    c = O.config(*cfg_tuple(f))
    n = f["cells"].shape[0]
    b = O.Batch(c, n)
    b.cells[:] = f["cells"]
    b.visits[:] = f["visits"].astype(np.int32)
    b.explored[:] = f["explored"]
    b.scal[:, :6] = f["scal"]
    obs_pre = b.obs()
    assert (obs_pre == f["obs_pre"]).all()
    obs, rew, te, tr = b.step(f["action"])
    assert (obs == f["obs"]).all()
    assert (rew == f["reward"]).all()
    assert (te == f["term"].astype(bool)).all()
    assert (tr == f["trunc"].astype(bool)).all()
    assert (b.cells == f["cells_post"]).all()
    assert (b.visits == f["visits_post"].astype(np.int32)).all()
    assert (b.explored == f["explored_post"]).all()
    sp = f["scal_post"]
    assert (b.scal[:, :6] == sp[:, :6]).all()
    for e in range(n):
        inf = b.info(e)
        assert inf[3] == sp[e, 6] and inf[4] == sp[e, 7] and inf[0] == sp[e, 8] and inf[1] == sp[e, 9]
    assert ((b.scal[:, O.S_POISONED] & 1).astype(bool) == f["root_raises"].astype(bool)).all()


@pytest.mark.parametrize("name", TRAJ_FILES)
def test_dummyvecenv_trajectories(name):
    """N envs sharing one global `random` stream, DummyVecEnv auto-reset order
    (A2C_training.py:216-218): terminal obs, reset obs, rewards, flags."""
    f = load(name)
    c = O.config(*cfg_tuple(f))
    acts = f["actions"]
    T, N = acts.shape
    mt = O.MT(int(f["seed"]))
    b = O.Batch(c, N)
    for e in range(N):
        b.reset_cpython(e, mt)
    assert (b.cells == f["maps0"]).all()
    assert (b.obs() == f["obs0"]).all()
    ri = 0
    for t in range(T):
        obs, rew, te, tr = b.step(acts[t])
        assert (rew == f["reward"][t]).all(), t
        assert (te == f["terminated"][t].astype(bool)).all(), t
        assert (tr == f["truncated"][t].astype(bool)).all(), t
        for e in range(N):
            if te[e] or tr[e]:
                assert (obs[e] == f["terminal_obs"][t, e]).all()
                b.reset_cpython(e, mt)
                assert f["reset_t"][ri] == t and f["reset_env"][ri] == e
                assert (b.cells[e] == f["reset_cells"][ri]).all()
                ri += 1
        assert (b.obs() == f["obs"][t]).all(), t
    assert ri == len(f["reset_t"])
    assert mt.u32() == f["next_u32"]


def test_lidar_first_hit_maps():
    """The (dx,dy) table reproduces the reference's per-ray first hit for a single
    obstacle at every window cell (includes (0,0) at r=1 and duplicate cells)."""
    f = np.load(__import__("golden_util").GOLDEN + "/lidar_firsthit.npz", allow_pickle=False)
    for key in f.files:
        C, R = (int(s[1:]) for s in key.split("_"))
        dx, dy = O.lidar_table(C, R)
        W = 2 * R + 1
        exp = f[key]
        got = np.zeros_like(exp)
        for cx in range(W):
            for cy in range(W):
                for i in range(C):
                    for r in range(1, R + 1):
                        if R + dx[i, r - 1] == cx and R + dy[i, r - 1] == cy:
                            got[cx * W + cy, i] = r
                            break
        assert (got == exp).all(), key


def test_survey_lidar_table_c16_r6():
    dx, dy = O.lidar_table(16, 6)
    assert list(zip(dx[2], dy[2])) == [(0, 0), (1, 1), (2, 2), (2, 2), (3, 3), (4, 4)]
    assert list(zip(dx[1], dy[1])) == [(0, 0), (1, 0), (2, 1), (3, 1), (4, 1), (5, 2)]
    assert list(zip(dx[8], dy[8])) == [(-r, 0) for r in range(1, 7)]


def test_philox_known_answer():
    """Random123 Philox4x32-10 KAT (counter=0,key=0 and the pi-digit vector)."""
    assert list(O.philox4x32([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(O.philox4x32([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(O.philox4x32([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_philox_reset_distribution_invariants():
    """Device-rng resets follow _generate_map's structure (plantos_env.py:338-372):
    border ring free, exactly P plants, rover on a free non-plant cell, visit/explored init."""
    c = O.config(20, 10, 12, 6, 16)
    n = 400
    b = O.Batch(c, n)
    thirsty = 0
    for e in range(n):
        b.reset_philox(e, 7, e, 0)
        cells = b.cells[e]
        assert (cells[0, :] != 1).all() and (cells[-1, :] != 1).all()
        assert (cells[:, 0] != 1).all() and (cells[:, -1] != 1).all()
        assert ((cells == 2) | (cells == 3)).sum() == 10
        thirsty += (cells == 3).sum()
        x, y = b.scal[e, :2]
        assert cells[x, y] == 0
        assert b.visits[e].sum() == 1 and b.visits[e, x, y] == 1
        assert b.explored[e, x, y] == 2 and (b.explored[e] > 0).sum() == 1
        assert b.scal[e, O.S_EPISODE] == 1
    frac = thirsty / (10 * n)
    assert 0.65 < frac < 0.75
