"""Gym facade for the env-level variants: the 4cars2 and stop ids build
with the reference's spaces, and their dynamics (device source on the CPU host-sim
backend) replay the reference's own trajectories (tests/golden/env_4cars2_*.npz,
env_stop_*.npz) step by step through reset()/step()."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _HostBackend:
    def __init__(self, variant, nb_car, nb_ped, nb_lines, seed):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools")])
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import hostsim
        self.h = hostsim.HostVec(variant, 1, nb_car, nb_ped, nb_lines, seed_base=seed)
        self.n_slots = 2 * nb_car if variant == "4cars2" else nb_car

    def reset(self, want_obs=True):
        return self.h.reset()

    def step(self, a):
        o, r, rl, d = self.h.step(np.asarray(a, dtype=np.float64))
        return o, r, rl, d

    def get_state(self):
        return self.h.state()


@pytest.mark.parametrize("name,gym_id", [("4cars2_412", "Crosswalk_hybrid_multi_coop_4cars2-v0"),
                                         ("stop_212", "Crosswalk_hybrid_multi_stop-v0")])
def test_facade_replays_reference(name, gym_id):
    from mhppo import envs
    g = np.load(os.path.join(ROOT, "tests", "golden", f"env_{name}.npz"))
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    be = _HostBackend(str(g["variant"]), nc, npd, nl, int(g["seed_base"]))
    env = envs.make(gym_id, car_b=None, ped_b=None, cross_b=None, nb_car=nc, nb_ped=npd, nb_lines=nl, dt=0.3,
                    max_episode=80, simulation="sin", backend=be)
    n_act = 4 * nc if name.startswith("4cars2") else 2 * nc
    assert env.action_space.shape == (n_act,)
    assert ("car_follow" in env.observation_space.keys()) == name.startswith("4cars2")
    state, _ = env.reset()
    np.testing.assert_array_equal(np.concatenate(list(state.values())), g["obs0"][0])
    for t in range(g["obs"].shape[1]):
        state, rew, done, trunc, _ = env.step(g["actions"][0, t])
        np.testing.assert_array_equal(np.concatenate(list(state.values())), g["obs"][0, t])
        np.testing.assert_array_equal(rew, g["rewards"][0, t])
        np.testing.assert_array_equal(env.reward_light, g["reward_light"][0, t])
        assert done == bool(g["done"][0, t])
    assert len(env.cars) == nc
