"""Host-side logic of the drop-in vec-env faces (plantos_amd.vec_env), on CPU.

The PlantOSBatch is replaced by tests/oracle_rollout.OracleBatch (the oracle with
the same interface), so this checks the adapter's own semantics -- SB3
DummyVecEnv auto-reset bookkeeping (terminal_observation, TimeLimit.truncated),
Monitor's info["episode"], PlantOSEnv._get_info keys (plantos_env.py:317-336),
lazy infos, gymnasium-0.29 final_observation/final_info -- without a GPU.
SB3 itself is not installed: DummyVecEnv's behaviour is restated from its
published semantics, parity unpinned against SB3 code.
"""
import numpy as np
import pytest

from oracle import oracle as O
from oracle_rollout import OracleBatch, OracleVec
from plantos_amd.vec_env import LazyInfos, PlantOSVecEnv, PlantOSVectorEnv, info_dict

CFG = dict(grid_size=7, num_plants=3, num_obstacles=3, lidar_range=3, lidar_channels=12)
INFO_KEYS = {"rover_position", "thirsty_plants", "hydrated_plants", "total_plants", "step_count", "explored_cells",
             "total_cells", "exploration_percentage", "lidar_range", "lidar_channels", "collided_with_wall",
             "total_collisions"}


def make(n, seed=5, max_steps=40):
    b = OracleBatch(n, seed=seed, max_steps=max_steps, **CFG)
    return PlantOSVecEnv(n, batch=b, max_steps=max_steps, **CFG)


def test_spaces_and_reset():
    v = make(6)
    assert v.observation_space.shape == (5 * 12 + 27,)
    assert v.action_space.n == 5
    obs = v.reset()
    assert obs.shape == (6, 87) and obs.dtype == np.float32
    assert set(v.reset_infos[0].keys()) == INFO_KEYS
    assert v.reset_infos[3]["step_count"] == 0 and v.reset_infos[3]["explored_cells"] == 1


def test_step_wait_matches_dummyvecenv_semantics():
    n, T, seed = 5, 95, 5
    v = make(n, seed)
    ref = OracleVec((7, 3, 3, 3, 12), np.arange(n), seed, max_steps=40)
    v.reset()
    ref_b = ref.b
    for e in range(n):
        ref_b.reset_philox(e, seed, e, 1)
    ref.ret[:] = 0
    rng = np.random.default_rng(1)
    seen_done = 0
    for t in range(T):
        a = rng.integers(0, 5, n)
        obs, rew, done, infos = v.step(a)
        # reference DummyVecEnv over the oracle: step, info of the final state, reset
        o, r, te, tr = ref_b.step(a)
        ref.ret += r
        pre = [ref_b.info(e) for e in range(n)]
        pre_sc = ref_b.scal.copy()
        rd = te | tr
        assert (rew == r.astype(np.float32)).all() and (done == rd).all()
        for e in range(n):
            d = infos[e]
            assert INFO_KEYS <= set(d.keys())
            th, hy, tot, ex, tc = pre[e]
            assert d["step_count"] == pre_sc[e, O.S_STEP] and d["explored_cells"] == ex
            assert d["total_cells"] == tc and d["thirsty_plants"] == th and d["hydrated_plants"] == hy
            assert d["rover_position"] == (pre_sc[e, O.S_X], pre_sc[e, O.S_Y])
            assert d["exploration_percentage"] == (np.float64(ex) / np.float64(tc)) * 100
            if rd[e]:
                seen_done += 1
                assert (d["terminal_observation"] == o[e]).all()
                assert d["TimeLimit.truncated"] == bool(tr[e] and not te[e])
                assert d["episode"]["l"] == pre_sc[e, O.S_STEP]
                assert d["episode"]["r"] == round(float(ref.ret[e]), 6)
                ref_b.reset_philox(e, seed, e, int(ref_b.scal[e, O.S_EPISODE]))
                ref.ret[e] = 0
            else:
                assert "terminal_observation" not in d and "episode" not in d
        o2 = o.copy()
        if rd.any():
            o2[rd] = ref_b.obs(np.nonzero(rd)[0])[rd]
        assert (obs == o2).all(), t
    assert seen_done >= n  # max_steps=40 over 95 steps: every env reset at least twice


def test_lazy_infos_build_on_demand():
    calls = []

    def build(i):
        calls.append(i)
        return {"i": i}

    li = LazyInfos(4, build)
    assert len(li) == 4 and calls == []
    assert li[2]["i"] == 2 and li[-1]["i"] == 3 and calls == [2, 3]
    assert [d["i"] for d in li] == [0, 1, 2, 3]
    assert calls == [2, 3, 0, 1]


def test_info_dict_percentage_is_float64():
    row = np.array([1, 2, 3, 4, 7, 9, 10, 375, 1, 5, 0], np.int32)
    d = info_dict(row, 6, 16)
    assert d["exploration_percentage"] == (np.float64(10) / np.float64(375)) * 100
    assert d["collided_with_wall"] is True and d["total_plants"] == 7


def test_get_set_attr_visit_counts_roundtrip():
    v = make(3)
    v.reset()
    vc = v.get_attr("visit_counts")
    assert len(vc) == 3 and vc[0].shape == (7, 7) and vc[0].sum() == 1
    vc[1][0, 0] = 9
    v.set_attr("visit_counts", [vc[1]], indices=[1])
    assert v.get_attr("visit_counts", 1)[0][0, 0] == 9
    assert v.get_attr("grid_size") == [7, 7, 7]
    pos = v.get_attr("rover_pos")
    assert all(0 <= x < 7 and 0 <= y < 7 for x, y in pos)
    plants = v.get_attr("plants", [0])[0]
    assert len(plants) == 3 and all(isinstance(t, bool) for t in plants.values())
    with pytest.raises(AttributeError):
        v.get_attr("nope")


def test_seed_and_methods():
    v = make(3)
    assert v.seed(11) == [11, 12, 13]
    assert v.env_is_wrapped(object) == [False] * 3
    with pytest.raises(NotImplementedError):
        v.render()


def test_gymnasium_vector_face():
    g = PlantOSVectorEnv(4, batch=OracleBatch(4, seed=2, max_steps=10, **CFG), max_steps=10, **CFG)
    obs, info = g.reset()
    assert obs.shape == (4, 87) and info == {}
    for t in range(10):
        obs, rew, term, trunc, infos = g.step(np.zeros(4, np.int64) + t % 5)
    assert trunc.all() and "final_observation" in infos
    assert infos["_final_observation"].all()
    assert infos["final_observation"][0].shape == (87,)
    assert "TimeLimit.truncated" not in infos["final_info"][0]


def test_stale_lazy_infos_fail_loudly():
    v = make(3)
    v.reset()
    _, _, _, infos1 = v.step(np.zeros(3, np.int64))
    d0 = infos1[0]  # read in time: served later from the host copy
    _, _, _, infos2 = v.step(np.zeros(3, np.int64))
    assert infos1[0] is d0 and infos1[1]["step_count"] == 1  # table fetched before expiry
    infos2[0]
    v.step(np.zeros(3, np.int64))
    with pytest.raises(RuntimeError):
        _ = [d for d in make(1).reset_infos]  # fresh env: fine
        infos2._build._info = None
        infos2[2]
