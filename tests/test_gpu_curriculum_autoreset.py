"""The batched CurriculumWrapper through the step kernels' OWN auto-resets (device-rng
maps: prefetched records, the wave-cooperative reset, the byte-coded 64x64 sector
kernel, the one-wave-per-env kernel), with desynchronized episodes, against the CPU
wrapper restatement that tests/test_oracle_curriculum.py pins to the reference's
classes (A2C_training.py:37-109: a threshold hit terminates; trainingCode.py:24-98:
it only marks the maze completed, 50 episodes per maze).  Every step: obs (incl. the
stale reset obs and carried visit slices), reward, terminated, truncated, terminal
obs; at the end: thresholds, counters, visit counts, cells, scalars."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from test_oracle_curriculum import OracleCurriculumVec

pytestmark = pytest.mark.gpu

CFG = {
    "g20": (20, 10, 12, 6, 16),       # pe_step_quad<C16,R6,1word> (f32 tile, prefetched records)
    "g64": (64, 100, 120, 6, 64),     # pe_step_quad<C64,R6> (byte-coded tile, LDS-DMA staged records)
    "g64r32": (64, 100, 120, 32, 64),  # pe_step_far
}


class PhiloxCurriculumVec(OracleCurriculumVec):
    """The same wrapper over the device-rng map stream: env e's k-th map is
    reset_philox(seed, e, k) (what pe_create / pe_reset / the auto-reset draw)."""

    def __init__(self, cfg, n, seed, **kw):
        super().__init__(cfg, n, 0, **kw)
        self.seed = seed
        for e in range(n):
            self.b.reset_philox(e, seed, e, 0)  # pe_create

    def _new_map(self, e):
        self.b.reset_philox(e, self.seed, e, int(self.b.scal[e, O.S_EPISODE]))


@pytest.mark.parametrize("variant", ["a2c", "trainingCode"])
@pytest.mark.parametrize("name,n,steps,spread,thr", [("g20", 1024, 90, 60, 3.0), ("g64", 160, 45, 30, 0.4),
                                                     ("g64r32", 128, 40, 25, 0.4)])
def test_curriculum_device_autoreset_matches_wrapper(name, n, steps, spread, thr, variant):
    from plantos_amd import PlantOSBatch
    G, P, Ob, R, C = cfg = CFG[name]
    seed = 41
    # low thresholds (percent explored) so that hits, terminating or not, happen in the window
    over = dict(initial_threshold=thr, threshold_increment=thr / 2)
    b = PlantOSBatch(n, grid_size=G, num_plants=P, num_obstacles=Ob, lidar_range=R, lidar_channels=C, seed=seed,
                     device="cuda:0")
    b.enable_curriculum(variant, **over)
    kw = dict(OracleCurriculumVec.VARIANTS["tc" if variant == "trainingCode" else "a2c"])
    kw.update(initial=over["initial_threshold"], inc=over["threshold_increment"])
    ov = PhiloxCurriculumVec(cfg, n, seed, **kw)
    assert (b.reset().cpu().numpy() == ov.reset()).all()
    start = (999 - np.random.default_rng(9).integers(0, spread, n)).astype(np.int32)
    sc = b.get_state(parts=("scalars",))["scalars"].cpu().numpy()
    sc[:, O.S_STEP] = start
    b.set_state(scalars=sc)
    ov.b.scal[:, O.S_STEP] = start
    act = torch.empty(n, dtype=torch.int32, device="cuda:0")
    hits = resets = 0
    for t in range(steps):
        b.synth_actions(seed, t, out=act)
        obs, rew, te, tr = b.step(act)
        o_obs, o_rew, o_te, o_tr, o_tobs = ov.step(act.cpu().numpy())
        assert (rew.cpu().numpy() == o_rew.astype(np.float32)).all(), t
        assert (te.cpu().numpy().astype(bool) == o_te).all() and (tr.cpu().numpy().astype(bool) == o_tr).all(), t
        done = o_te | o_tr
        if done.any():
            assert (b.terminal_obs.cpu().numpy()[done] == o_tobs[done]).all(), t
        assert (obs.cpu().numpy() == o_obs).all(), t
        hits += int(o_te.sum()) + int(ov.completed.sum())  # a2c: terminations; trainingCode: marks
        resets += int(done.sum())
    assert resets >= n and hits > 0
    thr, cnt = b.get_curriculum()
    assert (thr.cpu().numpy() == ov.thr).all()
    fin = np.stack([ov.episodes, ov.successes, ov.on_maze,
                    ov.completed.astype(int) | 2 * np.array([p is not None for p in ov.persistent])], 1)
    assert (cnt.cpu().numpy() == fin).all()
    st = b.get_state()
    assert (st["visits"].cpu().numpy() == ov.b.visits).all()
    assert (st["cells"].cpu().numpy() == ov.b.cells).all()
    assert (st["explored"].cpu().numpy() == ov.b.explored).all()
    b.close()
