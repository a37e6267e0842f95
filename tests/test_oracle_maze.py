"""The fork's maze map generator (gradio-app/plantos_env_new.py:355-358, 408-604)
against the reference itself: tests/golden/maze_*.npz hold consecutive reset()
layouts of the fork with map_generation_algo='maze' after random.seed(s)
(tools/gen_golden.py:gen_maze_maps), for meta grids of 1x1 .. 10x10 and the
fallback to the original generator when the maze has no room (maze_g7fallback).
Both CPU restatements are pinned: the oracle (oracle/plantos_oracle.c) and the
product's host-side seed-exact stream (csrc/pe_pystream.cpp, pe_pystream_*)."""
import glob
import os

import numpy as np
import pytest

from golden_util import GOLDEN, cfg_tuple, load
from oracle import oracle as O

MAZE_FILES = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "maze_*.npz")))


def test_fixtures_present():
    assert len(MAZE_FILES) >= 8


@pytest.mark.parametrize("name", MAZE_FILES)
def test_oracle_maze_matches_reference(name):
    f = load(name)
    cfg = O.config(*cfg_tuple(f), map_algo=1)
    b = O.Batch(cfg, 1)
    for si, s in enumerate(f["seeds"]):
        mt = O.MT(int(s))
        for k in range(f["cells"].shape[1]):
            b.reset_cpython(0, mt)
            assert (b.cells[0] == f["cells"][si, k]).all(), (name, si, k)
            assert tuple(b.scal[0, :2]) == tuple(f["rover"][si, k])
            assert (b.visits[0].sum(), b.visits[0][tuple(f["rover"][si, k])]) == (1, 1)
        assert mt.u32() == f["next_u32"][si]  # the exact number of MT draws consumed
    # the reset() obs of the first map
    b2 = O.Batch(cfg, 1)
    b2.reset_cpython(0, O.MT(int(f["seeds"][0])))
    assert (b2.obs() == f["obs0"][0]).all()


@pytest.mark.parametrize("name", MAZE_FILES)
def test_pystream_maze_matches_reference(name):
    from plantos_amd import _capi as C
    f = load(name)
    G, P, Ob, R, Cc = cfg_tuple(f)
    for si, s in enumerate(f["seeds"]):
        ps = C.PyStream(G, P, Ob, int(s), map_generation_algo="maze")
        cells, rover = ps.next(f["cells"].shape[1])
        assert (cells == f["cells"][si]).all() and (rover == f["rover"][si]).all(), (name, si)
        assert ps.getrandbits32() == f["next_u32"][si]
        ps.close()


def test_maze_needs_a_meta_grid():
    """G < 7: random.randint(0, -1) raises ValueError in the reference (:427)."""
    from plantos_amd import _capi as C
    with pytest.raises(ValueError):
        C.PyStream(6, 2, 3, 0, map_generation_algo="maze")
    b = O.Batch(O.config(6, 2, 3, 2, 8, map_algo=1), 1)
    assert O.lib().po_reset_cpython(O.ctypes.byref(b.cfg), O.ctypes.byref(O.MT(0).s), *[
        O._p(x) for x in (b.cells, b.visits, b.explored, b.scal)]) == -1


def test_philox_maze_is_a_maze():
    """Device-rng maze (the definition the GPU follows): every room centre of the
    3x3 meta grid carved, the 20x20 grid mostly but not fully open."""
    cfg = O.config(20, 10, 12, 6, 16, map_algo=1)
    b = O.Batch(cfg, 64)
    for e in range(64):
        b.reset_philox(e, 5, e, 0)
    c = b.cells
    assert (c[:, 3::6, 3::6][:, :3, :3] != 1).all()                       # every room centre open
    nfree = (c != 1).reshape(64, -1).sum(1)
    assert (nfree > 200).all() and (nfree < 400).all()
