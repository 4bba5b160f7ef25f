"""Deterministic evaluation oracle (oracle_eval_episode, restating Env_rollout.iterations
:152-252 as Algo_PPO.evaluate :738-747 runs it) vs the reference on its shipped weights
(tests/golden/eval_*.npz, made by tests/golden/gen/make_eval_golden.py).

Exact: the number of saves per env (including the scalable driver's every-step
re-decision when ped_traffic < nb_ped) and the pedestrians' waiting times.  Continuous
values within float32 noise: the reference's torch CPU Linear sums in another order than
the oracle's fmaf chain, a 1-ulp action difference the dynamics carry along (observed
max |d obs| 1.5e-5 on positions up to 1e3)."""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = ["coop_212", "naif_111", "scalable_211", "scalable_221"]
TOL = dict(obs=(1e-6, 1e-4), acts=(1e-6, 1e-4), rews_c=(1e-5, 1e-4), rews_d=(1e-5, 1e-4), waiting=(0, 1e-6))


def check_eval(out, g, env_slices=None):
    for k, (rt, at) in TOL.items():
        a, b = np.asarray(out[k], np.float64), np.asarray(g[k], np.float64)
        assert a.shape == b.shape, (k, a.shape, b.shape)
        np.testing.assert_allclose(a, b, rtol=rt, atol=at, err_msg=k)


@pytest.mark.parametrize("name", CASES)
def test_oracle_eval_matches_reference(name):
    import oracle
    g = np.load(os.path.join(ROOT, "tests", "golden", f"eval_{name}.npz"))
    E, K = len(g["n_obs"]), int(g["episodes"])
    res = oracle.evaluate(str(g["variant"]), int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                          [int(g["seed_base"]) + e for e in range(E)], K, g["w_cross"], g["w_wait"], g["w_choice"])
    for e, r in enumerate(res):
        assert len(r["rews_d"]) == g["n_rews_d"][e], (e, len(r["rews_d"]), g["n_rews_d"][e])
    check_eval({k: np.concatenate([r[k] for r in res]) for k in res[0]}, g)
