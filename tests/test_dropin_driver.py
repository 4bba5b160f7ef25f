"""Drop-in check: the reference's own training driver runs on the mhppo Gym facade.

The coop driver's classes (Coop-MH-PPO.ipynb cell 0: Model_PPO, Env_rollout,
Algo_PPO), AST-extracted and unmodified, train one iteration (batch_size=160 ->
2 episodes) twice: once on the reference env (Environments/Env_hybrid_multi_coop.py
under the gym stub) and once on `mhppo.envs.make(...)` whose backend is the
device env source compiled for the CPU (tools/hostsim.cpp; no GPU here).  Same
torch seed, same random stream => the collected batches and the updated weights
must be bit-identical.  Needs /root/reference (build container only); skipped
elsewhere.
"""
import contextlib
import io
import os
import random
import subprocess
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.isdir("/root/reference/Environments"),
                                reason="reference checkout not present")


class _HostBackend:
    def __init__(self, variant, nb_car, nb_ped, nb_lines, seed):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools")])
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import hostsim
        self.h = hostsim.HostVec(variant, 1, nb_car, nb_ped, nb_lines, seed_base=seed)

    def reset(self):
        return self.h.reset()

    def step(self, a):
        return self.h.step(np.asarray(a, dtype=np.float64))

    def get_state(self):
        return self.h.state()


def _train(env, nc, nl, npd, driver="coop"):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "gen"))
    import refclasses
    if driver == "coop":
        ns = refclasses.notebook_classes("coop", env=env, nb_lines=nl, nb_car=nc, nb_ped=npd)
        dc = 2 + 5 * (nc - 1) + 10
    else:  # Coop-MH-PPO-scalable.py (:1036-1052)
        ns = refclasses.scalable_classes(env=env, nb_lines=nl)
        dc = 2 + 6 * (2 * nl - 1) + 10
    torch.manual_seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        algo = ns["Algo_PPO"](ns["Model_PPO"], env, num_algo=100 * npd + 10 * nc + nl, num_states_c=13,
                              num_states_d=dc, num_actions=1, mean=-1.0, std=3.0, nb_cars=nc, dt=0.3,
                              batch_size=160)
        algo.train(1)
    ro = algo.rollout
    batch = [np.array(ro.batch_obs_cross + ro.batch_obs_wait), np.array(ro.batch_acts_cross + ro.batch_acts_wait),
             np.array(ro.batch_log_probs_cross + ro.batch_log_probs_wait), np.array(ro.batch_obs_choice)]
    weights = [p.detach().numpy().copy() for n in (algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice,
                                                    algo.critic_net_cross, algo.critic_net_choice)
               for p in n.parameters()]
    return batch, weights


def test_reference_driver_trains_on_facade_bit_identically(tmp_path, monkeypatch):
    (tmp_path / "load_model" / "parameters").mkdir(parents=True)
    monkeypatch.chdir(tmp_path)  # train() writes its reward curves there (:908-916)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "gen"))
    import refharness as R
    from mhppo import envs
    nc, npd, nl = 2, 1, 2
    random.seed(10)  # the reference module's import-time seed
    ref_env = R.make("coop", nc, npd, nl)
    with contextlib.redirect_stdout(io.StringIO()):
        b_ref, w_ref = _train(ref_env, nc, nl, npd)
    fac = envs.make("Crosswalk_hybrid_multi_coop-v0", car_b=R.CAR_B, ped_b=R.PED_B, cross_b=R.CROSS_B, nb_car=nc,
                    nb_ped=npd, nb_lines=nl, dt=0.3, max_episode=80, simulation="sin",
                    backend=_HostBackend("coop", nc, npd, nl, seed=10))
    assert fac.observation_space["car"].shape == ref_env.observation_space["car"].shape
    assert fac.observation_space["env"].shape == ref_env.observation_space["env"].shape
    assert fac.observation_space["ped"].shape == ref_env.observation_space["ped"].shape
    b_fac, w_fac = _train(fac, nc, nl, npd)
    for x, y in zip(b_ref, b_fac):
        assert np.array_equal(x, y)
    for x, y in zip(w_ref, w_fac):
        assert np.array_equal(x, y)


def test_scalable_driver_trains_on_facade_bit_identically(tmp_path, monkeypatch):
    """The same with Coop-MH-PPO-scalable.py's driver classes on the scalable env (ragged
    existing cars, `cars[i].exist` read by the rollout, :489-507), 4 slots, 2 pedestrians."""
    (tmp_path / "load_model" / "parameters").mkdir(parents=True)
    monkeypatch.chdir(tmp_path)
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden", "gen"))
    import refharness as R
    from mhppo import envs
    nc, npd, nl = 3, 2, 2
    random.seed(10)
    ref_env = R.make("scalable", nc, npd, nl)
    with contextlib.redirect_stdout(io.StringIO()):
        b_ref, w_ref = _train(ref_env, nc, nl, npd, driver="scalable")
    fac = envs.make("Crosswalk_hybrid_multi_coop_scalable-v0", car_b=R.CAR_B, ped_b=R.PED_B, cross_b=R.CROSS_B,
                    nb_car=nc, nb_ped=npd, nb_lines=nl, dt=0.3, max_episode=80, simulation="sin",
                    backend=_HostBackend("scalable", nc, npd, nl, seed=10))
    for k in ("car", "env", "ped"):
        assert fac.observation_space[k].shape == ref_env.observation_space[k].shape
    b_fac, w_fac = _train(fac, nc, nl, npd, driver="scalable")
    for x, y in zip(b_ref, b_fac):
        assert np.array_equal(x, y)
    for x, y in zip(w_ref, w_fac):
        assert np.array_equal(x, y)
