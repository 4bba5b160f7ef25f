"""Pin the C rollout oracle against the reference's own rollout collector.

Fixtures tests/golden/rollout_*.npz: Env_rollout.iterations_rand of the
reference drivers, run unmodified on recorded noise (make_rollout_golden.py).
Bucket membership and every discrete draw must match exactly; continuous
outputs to float32 tolerance (the oracle's MLP sums in a fixed fused-multiply-
add order, torch's CPU GEMV in another — last-bit differences).
"""
import glob
import os

import numpy as np
import pytest

import oracle
from rollout_util import bucket, returns

FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rollout_*.npz")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[8:-4] for f in FILES])
def test_oracle_rollout_matches_reference(path):
    g = np.load(path)
    v = str(g["variant"])
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    E = g["a_d"].shape[0]
    seeds = [int(g["seed_base"]) + e for e in range(E)]
    o = oracle.rollout(v, nc, npd, nl, seeds, g["w_cross"], g["w_wait"], g["w_choice"], forced_a=g["a_d"],
                       eps=g["eps"])
    b = bucket(o, v == "scalable")
    for k in ("obs_cross", "obs_wait", "obs_choice", "act_cross", "act_wait", "act_choice"):
        assert b[k].shape == g[k].shape, (k, b[k].shape, g[k].shape)
    np.testing.assert_array_equal(b["act_choice"], g["act_choice"])
    for k, tol in (("obs_cross", 2e-5), ("obs_wait", 2e-5), ("obs_choice", 2e-5), ("act_cross", 2e-5),
                   ("act_wait", 2e-5), ("logp_cross", 2e-5), ("logp_wait", 2e-5), ("logp_choice", 2e-5),
                   ("rew_cross", 1e-5), ("rew_wait", 1e-5), ("rew_choice", 1e-5)):
        np.testing.assert_allclose(b[k], g[k], rtol=tol, atol=tol, err_msg=k)
    for h in ("cross", "wait"):
        np.testing.assert_allclose(returns(b["rew_" + h]), g["ret_" + h], rtol=1e-4, atol=1e-4, err_msg=h)
    np.testing.assert_allclose(b["rew_choice"].astype(np.float32), g["ret_choice"], rtol=1e-5, atol=1e-5)
