"""GPU: the SB3-protocol drop-in (PlantOSVecEnv over the HIP batch) against the
same adapter over the oracle batch -- obs, rewards, dones and every info dict,
across auto-resets (terminal_observation, TimeLimit.truncated, episode)."""
import numpy as np
import pytest
import torch

from oracle_rollout import OracleBatch
from plantos_amd import PlantOSVecEnv, PlantOSVectorEnv

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n,T,max_steps", [
    (dict(grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16), 96, 130, 60),
    (dict(grid_size=25, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16), 70, 70, 30),
    (dict(grid_size=7, num_plants=3, num_obstacles=3, lidar_range=3, lidar_channels=12), 33, 50, 20),
])
def test_vec_env_gpu_vs_oracle(cfg, n, T, max_steps):
    seed = 21
    gpu = PlantOSVecEnv(n, seed=seed, max_steps=max_steps, device="cuda:0", **cfg)
    ref = PlantOSVecEnv(n, batch=OracleBatch(n, seed=seed, max_steps=max_steps, **cfg), max_steps=max_steps, **cfg)
    o1, o2 = gpu.reset(), ref.reset()
    assert (o1 == o2).all()
    for i in (0, n - 1):
        assert gpu.reset_infos[i] == ref.reset_infos[i]
    rng = np.random.default_rng(3)
    for t in range(T):
        a = rng.integers(0, 5, n)
        g_obs, g_rew, g_done, g_inf = gpu.step(a)
        r_obs, r_rew, r_done, r_inf = ref.step(a)
        assert (g_obs == r_obs).all() and (g_rew == r_rew).all() and (g_done == r_done).all(), t
        for e in list(np.nonzero(r_done)[0]) + [0, n // 2]:
            gd, rd = g_inf[e], r_inf[e]
            assert gd.keys() == rd.keys()
            for k in gd:
                if k == "terminal_observation":
                    assert (gd[k] == rd[k]).all()
                elif k == "episode":
                    assert gd[k]["r"] == rd[k]["r"] and gd[k]["l"] == rd[k]["l"]
                else:
                    assert gd[k] == rd[k], (t, e, k)
    assert gpu.get_attr("visit_counts", [5])[0].tolist() == ref.get_attr("visit_counts", [5])[0].tolist()
    gpu.close()


def test_host_faces_agree():
    """The numpy face with a pinned obs ring (host_buffers=3) and the zero-copy
    face (tensors=True, flags fetched lazily) return what the default numpy face
    returns, step for step, across auto-resets; ring arrays stay valid for 3 steps."""
    cfg = dict(grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16)
    n, seed, ms = 200, 5, 40
    envs = [PlantOSVecEnv(n, seed=seed, max_steps=ms, device="cuda:0", **cfg),
            PlantOSVecEnv(n, seed=seed, max_steps=ms, device="cuda:0", host_buffers=3, **cfg),
            PlantOSVecEnv(n, seed=seed, max_steps=ms, device="cuda:0", tensors=True, **cfg)]
    for v in envs:
        v.reset()
    rng = np.random.default_rng(8)
    kept = []
    for t in range(90):
        a = rng.integers(0, 5, n)
        out = [v.step(a if i < 2 else torch.as_tensor(a, device="cuda:0")) for i, v in enumerate(envs)]
        (o0, r0, d0, i0), (o1, r1, d1, i1), (o2, r2, d2, i2) = out
        o2, r2, d2 = o2.cpu().numpy(), r2.cpu().numpy(), d2.cpu().numpy()
        assert (o0 == o1).all() and (o0 == o2).all() and (r0 == r1).all() and (r0 == r2).all(), t
        assert (d0 == d1).all() and (d0 == d2).all() and r1.dtype == np.float32 and d1.dtype == bool
        for e in list(np.nonzero(d0)[0][:3]) + [1]:
            a0, a1, a2 = i0[e], i1[e], i2[e]
            assert a0.keys() == a1.keys() == a2.keys()
            if "terminal_observation" in a0:
                assert (a0["terminal_observation"] == a2["terminal_observation"]).all()
                assert a0["TimeLimit.truncated"] == a1["TimeLimit.truncated"] == a2["TimeLimit.truncated"]
                assert a0["episode"]["r"] == a2["episode"]["r"]
        kept.append((o1, o0.copy()))
        if len(kept) > 3:
            kept.pop(0)
        for ring_view, copy in kept:  # the last 3 ring arrays are intact
            assert (ring_view == copy).all()
    for v in envs:
        v.close()


def test_vec_env_tensor_mode_and_gym_face():
    cfg = dict(grid_size=20, num_plants=10, num_obstacles=12, lidar_range=6, lidar_channels=16)
    v = PlantOSVecEnv(64, tensors=True, device="cuda:0", **cfg)
    obs = v.reset()
    assert isinstance(obs, torch.Tensor) and obs.is_cuda and obs.shape == (64, 107)
    o, r, d, inf = v.step(torch.zeros(64, dtype=torch.int64, device="cuda:0"))
    assert o.is_cuda and r.dtype == torch.float32 and d.dtype == torch.bool
    v.close()
    g = PlantOSVectorEnv(8, max_steps=5, device="cuda:0", **cfg)
    g.reset(seed=3)
    for t in range(5):
        obs, rew, term, trunc, infos = g.step(np.full(8, t % 5))
    assert trunc.all() and infos["_final_info"].all()
    g.close()


@pytest.mark.parametrize("name", ["traj_g20_random", "traj_g20_explore", "traj_g7_explore", "traj_g21_explore"])
def test_cpython_mode_reproduces_reference_dummyvecenv(name):
    """reset_mode='cpython': the drop-in reproduces the REFERENCE's DummyVecEnv run
    end to end -- the layouts come from the product's own CPython-stream generator
    (random.seed(seed)), every obs / reward / done / terminal obs of every step
    equals the reference's (tests/golden/traj_*.npz)."""
    from golden_util import cfg_tuple, load
    f = load(name)
    G, P, O, R, C = cfg_tuple(f)
    T, N = f["actions"].shape
    v = PlantOSVecEnv(N, grid_size=G, num_plants=P, num_obstacles=O, lidar_range=R, lidar_channels=C,
                      device="cuda:0", reset_mode="cpython", python_seed=int(f["seed"]))
    obs = v.reset()
    assert (obs == f["obs0"]).all()
    for t in range(T):
        obs, rew, done, infos = v.step(f["actions"][t])
        assert (rew == f["reward"][t].astype(np.float32)).all(), t
        assert (done == (f["terminated"][t] | f["truncated"][t]).astype(bool)).all(), t
        for e in np.nonzero(done)[0]:
            assert (infos[e]["terminal_observation"] == f["terminal_obs"][t, e]).all(), (t, e)
        assert (obs == f["obs"][t]).all(), t
    v.close()


@pytest.mark.parametrize("name", ["curriculum_g20_explore", "curriculum_g7_explore", "curriculum_g20_random",
                                  "curriculum_tc_g20_explore", "curriculum_tc_g7_explore", "curriculum_tc_g20_random"])
def test_curriculum_reproduces_reference_wrapper(name):
    """PlantOSVecEnv(curriculum=True / "trainingCode", reset_mode='cpython') against the
    reference's CurriculumWrapper (A2C_training.py:37-109 / trainingCode.py:24-98) + env
    in a DummyVecEnv loop (tests/golden/curriculum_*.npz, curriculum_tc_*.npz):
    obs (incl. carried visit slices), rewards, curriculum terminations, terminal
    obs, per-step thresholds and the final wrapper counters."""
    from golden_util import cfg_tuple, load
    f = load(name)
    G, P, O, R, C = cfg_tuple(f)
    T, N = f["actions"].shape
    v = PlantOSVecEnv(N, grid_size=G, num_plants=P, num_obstacles=O, lidar_range=R, lidar_channels=C,
                      device="cuda:0", reset_mode="cpython", python_seed=int(f["seed"]),
                      curriculum="trainingCode" if "_tc_" in name else True)
    assert (v.reset() == f["obs0"]).all()
    for t in range(T):
        obs, rew, done, infos = v.step(f["actions"][t])
        assert (rew == f["reward"][t].astype(np.float32)).all(), t
        assert (done == (f["terminated"][t] | f["truncated"][t]).astype(bool)).all(), t
        for e in np.nonzero(done)[0]:
            assert (infos[e]["terminal_observation"] == f["terminal_obs"][t, e]).all(), (t, e)
        assert (obs == f["obs"][t]).all(), t
        if t % 25 == 0 or done.any():
            assert v.get_attr("exploration_threshold") == list(f["threshold"][t]), t
    thr, cnt = v.batch.get_curriculum()
    assert (cnt.cpu().numpy() == f["final_counters"]).all()
    vs = v.get_attr("visit_counts")
    assert [int(x.sum()) for x in vs] == list(f["visits_sum"][T - 1])
    v.close()
