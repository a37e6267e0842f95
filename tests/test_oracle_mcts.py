"""The MCTS restatement (oracle/plantos_mcts.c, test infrastructure) against the
reference's own searches: tests/golden/mcts_*.npz were produced by
mcts_custom_trainer.MCTS.search (:91-139) on the reference env
(tools/gen_golden.py:gen_mcts), recording the chosen action, the root's children
(action, visits, value in insertion order) and the np.random stream position +
CRC after every search.  Chains replay the reference's episodes decision by
decision with one continuing np.random stream."""
import zlib

import numpy as np
import pytest

from golden_util import cfg_tuple, load
from oracle import oracle as O

MCTS_FILES = ["mcts_g7", "mcts_g20", "mcts_g25", "mcts_g20d"]


def test_numpy_legacy_stream():
    """po_np_random / po_np_randint follow numpy's RandomState (seed, random, randint)."""
    for seed in (0, 7, 2**32 - 1):
        r = O.NpMT(seed)
        np.random.seed(seed)
        for t in range(2000):
            if t % 3 == 0:
                assert r.random() == np.random.random()
            else:
                n = 1 + t % 5
                assert r.randint(n) == np.random.randint(n)
        k, pos = r.state()
        st = np.random.get_state()
        assert pos == st[2] and (k == st[1]).all()


@pytest.mark.parametrize("name", MCTS_FILES)
def test_mcts_search_matches_reference(name):
    f = load(name)
    cfg = O.config(*cfg_tuple(f))
    ns, md, cp = int(f["n_sims"]), int(f["max_depth"]), float(f["c_param"])
    rng = None
    for i in range(len(f["action"])):
        if f["cseed"][i] >= 0:
            rng = O.NpMT(int(f["cseed"][i]))
        a, order, cv, cval = O.mcts_search(cfg, f["cells"][i], f["visits"][i], f["explored"][i], f["scal"][i],
                                           rng, ns, cp, md)
        assert a == f["action"][i], (name, i)
        np.testing.assert_array_equal(order, f["order"][i])
        np.testing.assert_array_equal(cv, f["cvisits"][i])
        np.testing.assert_array_equal(cval, f["cvalue"][i])  # f64 sums, bit-exact
        key, pos = rng.state()
        assert pos == f["pos_out"][i] and zlib.crc32(key.tobytes()) == f["crc_out"][i], (name, i)


def test_fixture_coverage():
    """The fixtures exercise what the device must reproduce: truncation inside the
    search (step counts at/after max_steps), fully-expanded roots, tiny grids."""
    g20 = load("mcts_g20")
    assert (g20["scal"][:, 2] >= 995).any()
    g7 = load("mcts_g7")
    assert (g7["order"] >= 0).all()  # every root fully expanded (n_sims >= 5)
    assert len(g7["action"]) > 100
