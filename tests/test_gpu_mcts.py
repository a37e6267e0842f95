"""GPU parity of the batched MCTS (pe_mcts_*, rl-env_amd/csrc/pe_mcts.hip).

Bar: bit-exact.  Every search must reproduce the reference's MCTS.search
(mcts_custom_trainer.py:91-139) as recorded in tests/golden/mcts_*.npz: the chosen
action, the root's children (action order, visits, f64 value sums) and the
np.random stream state after the search; chains replay the reference's episodes
decision by decision with the batch stepping the chosen actions in between.  At
the headline size (65536 envs) a sample of envs is checked against the oracle
(oracle/plantos_mcts.c) and every env against size-independent properties.
"""
import zlib

import numpy as np
import pytest
import torch

from golden_util import cfg_tuple, load
from oracle import oracle as O

pytestmark = pytest.mark.gpu

MCTS_FILES = ["mcts_g7", "mcts_g20", "mcts_g25", "mcts_g20d"]


def make(cfg, n, **kw):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = cfg
    return PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                        device="cuda:0", **kw)


def np_(t):
    return t.detach().cpu().numpy()


def same_stream(key_a, pos_a, key_b, pos_b, draws=700):
    """Two numpy MT states produce the same future draws."""
    ra, rb = np.random.RandomState(), np.random.RandomState()
    ra.set_state(("MT19937", np.asarray(key_a, np.uint32), int(pos_a), 0, 0.0))
    rb.set_state(("MT19937", np.asarray(key_b, np.uint32), int(pos_b), 0, 0.0))
    return (ra.randint(0, 2**32, draws, dtype=np.uint64) == rb.randint(0, 2**32, draws, dtype=np.uint64)).all()


@pytest.mark.parametrize("name", MCTS_FILES)
def test_mcts_matches_reference_searches(name):
    from plantos_amd.mcts import MCTS
    f = load(name)
    cfg = cfg_tuple(f)
    chains = np.unique(f["chain"])
    rows = [np.nonzero(f["chain"] == c)[0] for c in chains]
    n = len(chains)
    b = make(cfg, n, autoreset=False)
    first = np.array([r[0] for r in rows])
    scal = np.zeros((n, 8), np.int32)
    scal[:, :6] = f["scal"][first]
    b.set_state(cells=f["cells"][first], visits=f["visits"][first], explored=f["explored"][first], scalars=scal)
    m = MCTS(b, n_simulations=int(f["n_sims"]), c_param=float(f["c_param"]), max_depth=int(f["max_depth"]),
             seed=f["cseed"][first].astype(np.uint32))
    depth = max(len(r) for r in rows)
    for d in range(depth):
        live = np.array([len(r) > d for r in rows])
        idx = np.array([r[d] if len(r) > d else r[0] for r in rows])
        if d > 0:  # the live state must be the reference's state before decision d
            st = b.get_state()
            assert (np_(st["cells"])[live] == f["cells"][idx][live]).all(), (name, d)
            assert (np_(st["visits"])[live] == f["visits"][idx][live]).all(), (name, d)
        a, order, cv, cval = m.search(mask=live, root_stats=True)
        torch.cuda.synchronize()
        a, order, cv, cval = np_(a), np_(order), np_(cv), np_(cval)
        assert (a[live] == f["action"][idx][live]).all(), (name, d, a[live], f["action"][idx][live])
        assert (order[live] == f["order"][idx][live]).all(), (name, d)
        assert (cv[live] == f["cvisits"][idx][live]).all(), (name, d)
        assert (cval[live] == f["cvalue"][idx][live]).all(), (name, d)  # f64 sums, bit-exact
        key, pos = m.get_rng_state()
        for k in np.nonzero(live)[0]:
            i = idx[k]
            if pos[k] == f["pos_out"][i]:
                assert zlib.crc32(key[k].tobytes()) == f["crc_out"][i], (name, d, k)
            else:  # numpy reports pos 624 over the untwisted words at a round boundary
                assert f["pos_out"][i] == 624 and pos[k] == 0, (name, d, k, pos[k], f["pos_out"][i])
        step_a = np.where(live, a, 4).astype(np.int32)
        b.step(torch.as_tensor(step_a, device="cuda:0"))
    m.close()
    b.close()


def test_rng_state_round_trip():
    from plantos_amd.mcts import MCTS
    n = 70
    b = make((20, 10, 12, 6, 16), n)
    m = MCTS(b, n_simulations=5, max_depth=10, seed=3)
    key0, pos0 = m.get_rng_state()
    for e in (0, 1, n - 1):
        np.random.seed(3 + e)
        st = np.random.get_state()
        assert same_stream(key0[e], pos0[e], st[1], st[2])
    rs = np.random.RandomState(11)
    keys = np.zeros((n, 624), np.uint32)
    poss = np.zeros(n, np.int32)
    for e in range(n):
        r = np.random.RandomState(1000 + e)
        r.randint(0, 2**32, int(rs.randint(0, 2000)), dtype=np.uint64)
        st = r.get_state()
        keys[e], poss[e] = st[1], st[2]
    poss[0] = 0
    poss[1] = 1
    poss[2] = 623
    m.set_rng_state(keys, poss)
    k2, p2 = m.get_rng_state()
    for e in range(n):
        if poss[e] not in (0, 624):
            assert p2[e] == poss[e] and (k2[e] == keys[e]).all(), e
        assert same_stream(k2[e], p2[e], keys[e], poss[e]), e
    # a search advances every stream exactly as the oracle's
    m.search()
    torch.cuda.synchronize()
    st = b.get_state()
    cells, visits, expl, sc = (np_(st[k]) for k in ("cells", "visits", "explored", "scalars"))
    cfg = O.config(20, 10, 12, 6, 16)
    k3, p3 = m.get_rng_state()
    for e in (0, 1, 2, 5, n - 1):
        r = O.NpMT(0)
        r.s.mt[:] = keys[e].tolist()
        r.s.index = int(poss[e])
        O.mcts_search(cfg, cells[e], visits[e], expl[e], sc[e], r, 5, 1.414, 10)
        kk, pp = r.state()
        assert same_stream(k3[e], p3[e], kk, pp), e
    m.close()
    b.close()


def test_headline_size_search():
    """65536 envs, train_mcts settings (n_sims 50, max_depth 100): properties on
    every env, the oracle on a sample."""
    from plantos_amd.mcts import MCTS
    n = 65536
    cfgt = (20, 10, 12, 6, 16)
    b = make(cfgt, n, seed=5)
    acts = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(37):  # move the envs off their reset states
        b.step(b.synth_actions(5, t, out=acts))
    m = MCTS(b, n_simulations=50, max_depth=100, seed=123)
    st = b.get_state()
    cells, visits, expl, sc = (np_(st[k]) for k in ("cells", "visits", "explored", "scalars"))
    a, order, cv, cval = m.search(root_stats=True)
    torch.cuda.synchronize()
    a, order, cv, cval = np_(a), np_(order), np_(cv), np_(cval)
    assert ((a >= 0) & (a <= 4)).all()
    assert (cv.sum(1) == 50).all()                     # every simulation backs up through one root child
    assert (np.sort(order, 1) == np.arange(5)).all()    # all 5 actions expanded (n_sims >= 5)
    # the live env state is untouched by the search
    st2 = b.get_state()
    assert (np_(st2["visits"]) == visits).all() and (np_(st2["cells"]) == cells).all()
    cfg = O.config(*cfgt)
    rng = np.random.default_rng(0)
    for e in np.concatenate([[0, 1, n - 1], rng.choice(n, 29, replace=False)]):
        r = O.NpMT(123 + int(e))
        oa, oo, ocv, ocval = O.mcts_search(cfg, cells[e], visits[e], expl[e], sc[e], r, 50, 1.414, 100)
        assert oa == a[e] and (oo == order[e]).all() and (ocv == cv[e]).all() and (ocval == cval[e]).all(), e
    m.close()
    b.close()


def test_masked_search_leaves_other_envs():
    from plantos_amd.mcts import MCTS
    n = 130
    b = make((7, 3, 3, 3, 12), n, seed=2)
    m = MCTS(b, n_simulations=8, max_depth=12, seed=0)
    key0, pos0 = m.get_rng_state()
    m.actions.fill_(-7)
    mask = np.zeros(n, np.uint8)
    mask[::3] = 1
    a = np_(m.search(mask=mask))
    key1, pos1 = m.get_rng_state()
    off = mask == 0
    assert (a[off] == -7).all() and ((a[~off] >= 0) & (a[~off] <= 4)).all()
    assert (pos1[off] == pos0[off]).all() and (key1[off] == key0[off]).all()
    assert (pos1[~off] != pos0[~off]).any()
    m.close()
    b.close()


def test_mcts_drives_the_vec_env():
    """INTEGRATION.md's loop: MCTS over a PlantOSVecEnv, actions stepped on the device."""
    from plantos_amd import PlantOSVecEnv
    from plantos_amd.mcts import MCTS
    env = PlantOSVecEnv(16, grid_size=25, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16,
                        tensors=True, device="cuda:0", seed=4)
    mcts = MCTS(env, n_simulations=12, c_param=1.414, max_depth=20, seed=0)
    cfg = O.config(25, 10, 12, 6, 16)
    streams = {e: O.NpMT(e) for e in (0, 7, 15)}  # env e: np.random.seed(0 + e), continuing across decisions
    obs = env.reset()
    for _ in range(5):
        st = env.batch.get_state()
        actions = mcts.search(obs)
        torch.cuda.synchronize()
        a = np_(actions).copy()
        cells, visits, expl, sc = (np_(st[k]) for k in ("cells", "visits", "explored", "scalars"))
        for e, r in streams.items():
            assert O.mcts_search(cfg, cells[e], visits[e], expl[e], sc[e], r, 12, 1.414, 20)[0] == a[e]
        obs, rew, dones, infos = env.step(actions)
        assert ((a >= 0) & (a <= 4)).all()
    env.close()
