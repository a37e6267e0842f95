"""GPU parity of the fork's maze generator (map_generation_algo='maze',
gradio-app/plantos_env_new.py:408-604) as a device reset: device-rng maze resets
vs the oracle's definition (po_reset_philox, map_algo=1), rollouts with auto-reset
vs the oracle every step, and the seed-exact CPython mode vs the reference's own
maze layouts (tests/golden/maze_*.npz)."""
import numpy as np
import pytest
import torch

from golden_util import cfg_tuple, load
from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu

CFG = {
    "g20": (20, 10, 12, 6, 16),
    "g25": (25, 10, 12, 6, 16),
    "g64": (64, 100, 120, 6, 64),
    "g7": (7, 3, 3, 3, 12),
    "g7fallback": (7, 30, 3, 3, 12),
    "g13": (13, 5, 6, 3, 12),
}


def make(cfg, n, **kw):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = cfg
    return PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                        device="cuda:0", map_generation_algo="maze", **kw)


def np_(t):
    return t.detach().cpu().numpy()


@pytest.mark.parametrize("name", list(CFG))
def test_device_maze_reset_matches_oracle(name):
    cfg = CFG[name]
    n = 512 if cfg[0] <= 32 else 96
    b = make(cfg, n, seed=99)
    st = {k: np_(v) for k, v in b.get_state().items()}
    ob = O.Batch(O.config(*cfg, map_algo=1), n)
    for e in range(n):
        ob.reset_philox(e, 99, e, 0)
    assert (st["cells"] == ob.cells).all()
    assert (st["visits"] == ob.visits).all()
    assert (st["scalars"] == ob.scal).all()
    assert (np_(b.reset(mask=np.zeros(n, np.uint8))) == ob.obs()).all()
    b.close()


@pytest.mark.parametrize("name,n,steps", [("g20", 2048, 1050), ("g7fallback", 300, 1010), ("g64", 128, 60)])
def test_maze_rollout_parity(name, n, steps):
    """Auto-reset inside the step kernel generates mazes (the 1000-step truncation
    is crossed): every output of every step vs the oracle."""
    cfg = CFG[name]
    seed = 31
    b = make(cfg, n, seed=seed)
    ov = OracleVec(cfg, np.arange(n), seed, map_algo=1)
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        o_obs, o_rew, o_te, o_tr, o_tobs, o_ret, o_len = ov.step(np_(act))
        assert (np_(rew) == o_rew.astype(np.float32)).all(), t
        assert (np_(te).astype(bool) == o_te).all() and (np_(tr).astype(bool) == o_tr).all(), t
        assert (np_(obs) == o_obs).all(), t
    st = b.get_state()
    assert (np_(st["cells"]) == ov.b.cells).all()
    assert (np_(st["scalars"]) == ov.b.scal).all()
    b.close()


@pytest.mark.parametrize("name", ["maze_g20", "maze_g25", "maze_g7fallback"])
def test_cpython_maze_layouts_on_device(name):
    """reset_mode='cpython' + maze: the vec env's envs start on the reference's own
    maze layouts (DummyVecEnv order: env k gets the k-th reset of the stream)."""
    from plantos_amd import PlantOSVecEnv
    f = load(name)
    G, P, Ob, R, C = cfg_tuple(f)
    k = f["cells"].shape[1]
    env = PlantOSVecEnv(k, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C,
                        reset_mode="cpython", python_seed=int(f["seeds"][0]), map_generation_algo="maze",
                        device="cuda:0")
    obs = env.reset()
    st = env.batch.get_state()
    assert (np_(st["cells"]) == f["cells"][0]).all()
    assert (np_(st["scalars"])[:, :2] == f["rover"][0]).all()
    assert (np.asarray(obs)[0] == f["obs0"][0]).all()
    env.close()


def test_maze_small_grid_rejected():
    from plantos_amd import _capi as C
    with pytest.raises(ValueError):
        make((6, 2, 3, 2, 8), 4)
    assert C.PE_MAP_MAZE == 1
