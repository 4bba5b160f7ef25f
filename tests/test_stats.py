"""get_average (Coop-MH-PPO-scalable.py:1550-1675) ported as mhppo.stats.get_average, pinned
against the reference function itself run on the reference's own evaluation trajectories
(tests/golden/stats_*.npz, made by tests/golden/gen/make_stats_golden.py from
tests/golden/eval_*.npz).  Shares and counts exact; float32 torch statistics equal to the
reference's (same torch reductions on the same values in the same order, CPU); NaN / inf
where the reference has them (e.g. a non-existent car's speed 0 makes (25 - Sc)/Vc
infinite, :1619)."""
import glob
import os

import numpy as np
import pytest
import torch

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(G, "stats_*.npz")))
KEYS_SKIP = {"variant", "nb_car", "nb_ped", "nb_lines", "eval_fixture"}


def _check(got, g, rtol):
    for k in g.files:
        if k in KEYS_SKIP:
            continue
        ref = float(g[k])
        val = got[k]
        if np.isnan(ref):
            assert np.isnan(val), (k, val)
        elif np.isinf(ref):
            assert val == ref, (k, val, ref)
        else:
            assert abs(val - ref) <= rtol * max(1.0, abs(ref)), (k, val, ref)


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[6:-4] for f in FILES])
def test_get_average_matches_reference(path):
    from mhppo.stats import get_average
    g = np.load(path)
    ev = np.load(os.path.join(G, str(g["eval_fixture"])))
    got = get_average(torch.tensor(ev["obs"]), str(g["variant"]), int(g["nb_car"]), int(g["nb_ped"]),
                      int(g["nb_lines"]))
    # episodes = runs of equal cross (:1593): the choix scenario fixes cross = 3 in every episode,
    # so the reference's loop sees one long run there
    n_ep = int(ev["episodes"]) * len(ev["n_obs"])
    assert got["episodes"] == (1 if "choix" in path else n_ep)
    _check(got, g, 1e-6)
