"""Pin the C env oracle against golden vectors captured from the reference itself.

Fixtures: tests/golden/env_*.npz, produced by tests/golden/gen/make_env_golden.py
which runs /root/reference/Environments/*.py (under an offline gym stub) with one
CPython random stream per env.  Equality is bit-exact on every recorded field:
flat obs (float32), rewards and reward_light (float64), done, the RNG cursor
after reset and every step, the internal pedestrian/car state, and the final
MT19937 state.
"""
import glob
import os

import numpy as np
import pytest

from oracle import OracleEnv

FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "env_*.npz")))


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[4:-4] for f in FILES])
def test_oracle_matches_reference(path):
    g = np.load(path)
    v = str(g["variant"])
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    E, T = g["obs"].shape[:2]
    for e in range(E):
        env = OracleEnv(v, nc, npd, nl, seed=int(g["seed_base"]) + e)
        o = env.reset()
        assert np.array_equal(o, g["obs0"][e]), f"reset obs env {e}"
        assert env.rng_state()[1] % 624 == g["mti0"][e] % 624
        for t in range(T):
            o, r, rl, d = env.step(g["actions"][e, t])
            ctx = f"env {e} step {t}"
            assert np.array_equal(o, g["obs"][e, t]), ctx
            assert np.array_equal(r, g["rewards"][e, t]), ctx
            assert np.array_equal(rl, g["reward_light"][e, t]), ctx
            assert d == bool(g["done"][e, t]), ctx
            assert env.rng_state()[1] % 624 == g["mti"][e, t] % 624, ctx
            assert np.array_equal(env.dump(), g["dump"][e, t]), ctx
        mt, _ = env.rng_state()
        assert np.array_equal(mt, g["final_mt"][e])


def test_episode_is_80_steps():
    g = np.load(FILES[0])
    assert g["done"].shape[1] == 80 and g["done"][:, -1].all() and not g["done"][:, :-1].any()
