"""The Gym facade (mhppo.envs.make, Environments/__init__.py:3-42) on its DEFAULT backend —
a one-env VecCrosswalk on the GPU — replays the reference's own trajectories
(tests/golden/env_*.npz, env 0 of each, on random.seed(seed_base)) through the reference
surface: reset() -> (OrderedDict, {}), step(a) -> (state, rewards, done, False, {}),
reward_light, cars[i] / pedestrian[j] attributes, observation/action spaces."""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "env_*.npz")))
IDS = {"coop": "Crosswalk_hybrid_multi_coop-v0", "4cars": "Crosswalk_hybrid_multi_coop_4cars-v0",
       "scalable": "Crosswalk_hybrid_multi_coop_scalable-v0", "naif": "Crosswalk_hybrid_multi_naif-v0",
       "4cars2": "Crosswalk_hybrid_multi_coop_4cars2-v0", "stop": "Crosswalk_hybrid_multi_stop-v0"}
CAR_B = np.array([[-4.0, 10.], [2.0, 10.]])
PED_B = np.array([[-0.05, 0.75, 0.0, -3.0], [0.05, 1.75, 4., -0.5]])
CROSS_B = np.array([2.5, 3.0])


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[4:-4] for f in FILES])
def test_gpu_facade_replays_reference(path):
    from mhppo import envs
    g = np.load(path)
    v = str(g["variant"])
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    env = envs.make(IDS[v], car_b=CAR_B, ped_b=PED_B, cross_b=CROSS_B, nb_car=nc, nb_ped=npd, nb_lines=nl, dt=0.3,
                    max_episode=80, simulation="sin", seed=int(g["seed_base"]))
    assert env.venv.device.type == "cuda"
    state, info = env.reset()
    assert info == {} and list(state.keys()) == sorted(state.keys())
    np.testing.assert_array_equal(np.concatenate(list(state.values())), g["obs0"][0])
    k = g["dump"].shape[2]
    for t in range(g["obs"].shape[1]):
        state, rew, done, trunc, info = env.step(g["actions"][0, t])
        assert trunc is False and info == {}
        np.testing.assert_allclose(np.concatenate(list(state.values())), g["obs"][0, t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(rew, g["rewards"][0, t], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(env.reward_light, g["reward_light"][0, t], rtol=1e-9, atol=1e-12)
        assert done == bool(g["done"][0, t])
        dump = g["dump"][0, t]
        for j, p in enumerate(env.pedestrian):  # the attribute view the drivers read
            assert p.waiting_time == pytest.approx(dump[20 * j + 12], rel=1e-9, abs=1e-12)
            assert p.decision == dump[20 * j + 4]
        for i, c in enumerate(env.cars[:(k - 20 * npd) // 8]):
            assert c.exist == bool(dump[20 * npd + 8 * i + 7])
