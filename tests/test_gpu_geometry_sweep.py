"""A seeded sweep of geometries through every step kernel the library selects: the
runtime-(C, R) sector kernel (4 <= C <= 64, 2 <= R <= 14, one-word and multi-word
rows; a byte-coded obs tile above 32 rays), the compile-time sector kernels, and the
one-wave-per-env kernel (C > 64, R > 14 or R = 1) -- each against the oracle
(plantos_env.py:160-315 restated), every output of every step, episodes
desynchronized so that auto-resets happen inside the window, the final state
included.  Batch sizes are ragged (a partial last workgroup).  A second sweep covers
33 <= C <= 64 (round 4: the byte-coded runtime sector kernel) and the byte-coded
obs boundary (obs_codes) on runtime-sector geometries; a third (round 5) the long ranges
R in {16, 20, 32}, C = 64 / R = 32 through the far sector kernel (pe_step_far) where it
applies.  The verdict's R > 14 sweep case."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle_rollout import OracleVec

pytestmark = pytest.mark.gpu


def _geometries():
    rng = np.random.default_rng(2026)
    out = []
    while len(out) < 14:
        kind = len(out) % 3
        if kind < 2:  # the runtime sector kernel's range
            C, R = int(rng.integers(4, 33)), int(rng.integers(2, 15))
        else:         # the wave kernel's
            if rng.random() < 0.5:
                C, R = int(rng.integers(33, 100)), int(rng.integers(1, 12))
            else:
                C, R = int(rng.integers(4, 40)), int(rng.integers(15, 30))
        G = int(rng.integers(5, 41))
        cells = G * G
        O_ = int(rng.integers(0, max(1, cells // 10)))
        P = int(rng.integers(1, max(2, min(40, cells // 8))))
        # map generation needs room: clusters of <= 9 cells, P plants + the rover
        if (O_ // 3) * 9 + P + 1 > cells - 4 * G:
            continue
        out.append((G, P, O_, R, C))
    return out


def _wide_geometries():
    """33 <= C <= 64, 2 <= R <= 14 (the byte-coded runtime sector kernel)"""
    rng = np.random.default_rng(4044)
    out = []
    while len(out) < 10:
        C, R = int(rng.integers(33, 65)), int(rng.integers(2, 15))
        G = int(rng.integers(5, 49))
        cells = G * G
        O_ = int(rng.integers(0, max(1, cells // 10)))
        P = int(rng.integers(1, max(2, min(40, cells // 8))))
        if (O_ // 3) * 9 + P + 1 > cells - 4 * G:
            continue
        out.append((G, P, O_, R, C))
    return out


GEOS = _geometries()
WIDE = _wide_geometries()
# long ranges (R > 14, round 5): C = 64 / R = 32 at G in [33, 64] runs the far sector
# kernel (pe_step_far, compile-time rays, G + 2R in (96, 128]); R = 16 / 20 and G
# outside that range the one-wave-per-env kernel
FAR = [(64, 100, 120, 32, 64), (40, 30, 40, 32, 64), (33, 12, 20, 32, 64), (21, 8, 10, 32, 64),
       (48, 40, 60, 16, 64), (24, 10, 12, 20, 16)]


def _far_kernel(G, R, C):
    return C == 64 and R == 32 and 96 < G + 2 * R <= 128


def _ids(geos):
    return [f"G{g}P{p}O{o}R{r}C{c}" for g, p, o, r, c in geos]


# (round 6) runtime-sector geometries whose uneven compass sectors span more than 15 rows at
# long range: those sectors take the LDS-table rays, the others the register window
# (pe_quad.hpp quad_rays_rt_reg), in one launch -- C = 5 / 9 / 10 at R = 13 / 14
MIXED = [(20, 8, 16, 14, 5), (23, 10, 20, 13, 9), (28, 12, 24, 14, 10)]


@pytest.mark.parametrize("cfg", GEOS + WIDE + FAR + MIXED, ids=_ids(GEOS) + _ids(WIDE) + _ids(FAR) + _ids(MIXED))
def test_geometry_sweep_parity(cfg):
    _sweep(cfg, codes=False)


# the byte-coded obs boundary on runtime-sector geometries (f32 and byte tiles) and the
# far sector kernel
CODES = [g for g in GEOS if 4 <= g[4] <= 64 and 2 <= g[3] <= 14][:3] + WIDE[:3] + FAR[:2]


@pytest.mark.parametrize("cfg", CODES, ids=_ids(CODES))
def test_geometry_sweep_codes_parity(cfg):
    _sweep(cfg, codes=True)


def _sweep(cfg, codes):
    from plantos_amd import PlantOSBatch
    G, P, O_, R, C = cfg
    n, steps, seed = 133, 60, 17
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=O_, lidar_range=R, lidar_channels=C, seed=seed,
                     device="cuda:0", obs_codes=codes)
    rt = 4 <= C <= 64 and 2 <= R <= 14
    if rt:  # (or a compile-time specialization of the same sector kernel)
        assert b.kernel_name.startswith("pe_step_quad"), b.kernel_name
    elif _far_kernel(G, R, C):
        assert b.kernel_name == "pe_step_far<C64,R32,bytetile>", b.kernel_name
    elif C > 64 or R > 14:
        assert b.kernel_name == "pe_step_wave", b.kernel_name
    f32 = torch.empty((n, b.obs_dim), dtype=torch.float32, device="cuda:0")
    ov = OracleVec(cfg, np.arange(n), seed)
    start = (999 - np.random.default_rng(3).integers(0, 40, n)).astype(np.int32)
    sc = b.get_state(parts=("scalars",))["scalars"].cpu().numpy()
    sc[:, O.S_STEP] = start
    b.set_state(scalars=sc)
    ov.b.scal[:, O.S_STEP] = start
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        if codes:
            obs = b.expand_codes(b.io, 1, f32)[0]
        o_obs, o_rew, o_te, o_tr, o_tobs, o_ret, o_len = ov.step(act.cpu().numpy())
        assert (rew.cpu().numpy() == o_rew.astype(np.float32)).all(), t
        assert (te.cpu().numpy().astype(bool) == o_te).all() and (tr.cpu().numpy().astype(bool) == o_tr).all(), t
        assert (obs.cpu().numpy() == o_obs).all(), t
        done = o_te | o_tr
        if done.any():
            assert (b.terminal_obs.cpu().numpy()[done] == o_tobs[done]).all(), t
            assert (b.episode_return.cpu().numpy()[done] == o_ret[done]).all(), t
    st = b.get_state()
    assert (st["cells"].cpu().numpy() == ov.b.cells).all()
    assert (st["visits"].cpu().numpy() == ov.b.visits).all()
    assert (st["scalars"].cpu().numpy() == ov.b.scal).all()
    b.close()
