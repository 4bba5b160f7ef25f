"""The device env source (mh-ppo_amd/csrc/env_body.h), compiled for the CPU by
tools/hostsim.cpp, reproduces the reference fixtures bit-exactly.

With host libm (glibc, what CPython uses) there is no transcendental ULP gap,
so this pins the kernel's LOGIC: RNG draw order, branch structure, Python
min/max/floordiv semantics.  The GPU test (test_env_gpu.py) then only has to
account for device-libm ULPs.
"""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "env_*.npz")))


@pytest.fixture(scope="module")
def hostsim():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools")])
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import hostsim as hs
    return hs


# view: the step on the register env view (where compiled: single-pedestrian fixture shapes)
# or forced onto the generic in-HBM view (MHPPO_GENERIC_STEP)
@pytest.mark.parametrize("view", ["default", "generic"])
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[4:-4] for f in FILES])
def test_device_source_matches_reference(hostsim, path, view):
    g = np.load(path)
    E, T = g["obs"].shape[:2]
    h = hostsim.HostVec(str(g["variant"]), E, int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                        seed_base=int(g["seed_base"]), flags=2 if view == "generic" else 0)
    assert np.array_equal(h.reset(), g["obs0"])
    k = g["dump"].shape[2]
    for t in range(T):
        o, r, rl, d = h.step(g["actions"][:, t])
        assert np.array_equal(o, g["obs"][:, t]), t
        assert np.array_equal(r, g["rewards"][:, t]), t
        assert np.array_equal(rl, g["reward_light"][:, t]), t
        assert np.array_equal(d, g["done"][:, t]), t
        assert np.array_equal(h.state()[:, :k], g["dump"][:, t]), t


@pytest.mark.parametrize("shape", [(2, 1, 1), (4, 2, 2), (8, 1, 4)])
def test_device_choix_test_matches_oracle(hostsim, shape):
    """choix_test (:629-633) + get_state, then 80 steps: the device source on the CPU
    equals the C oracle bit for bit (observations, rewards, reward_light)."""
    import oracle
    nc, npd, nl = shape
    N = 6
    h = hostsim.HostVec("scalable", N, nc, npd, nl, seed_base=515)
    orc = [oracle.OracleEnv("scalable", nc, npd, nl, seed=515 + e) for e in range(N)]
    assert np.array_equal(h.reset(), np.stack([o.reset() for o in orc]))
    assert np.array_equal(h.choix_test(), np.stack([o.choix_test() for o in orc]))
    S = 2 * nl
    rng = np.random.default_rng(1)
    for t in range(80):
        a = np.concatenate([rng.uniform(-4, 2, (N, S)), np.where(rng.random((N, S)) < 0.5, -1.0, 1.0)], 1)
        hs = h.step(a)
        os_ = [o.step(a[e]) for e, o in enumerate(orc)]
        for j in range(3):
            assert np.array_equal(hs[j], np.stack([x[j] for x in os_])), (t, j)
