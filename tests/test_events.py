"""Per-env event counters (SURVEY §5 Metrics): the reference env's only run-time diagnostics
are five prints inside pedestrian.detection ("Accident! : ", "Possible accident! ", "Small
mistake - priority ? ", "Pedestrian is not waiting ", "Mauvais signal vert ";
Env_hybrid_multi_coop_scalable.py:186, 200, 222, 227, 236; 4cars :293-334; naif :189-233).
The build counts them per env instead of printing.

Pinned against tests/golden/events_<name>.npz: the reference envs' own stdout, captured per env
and step on the trajectories of tests/golden/env_<name>.npz (tests/golden/gen/
make_events_golden.py).  Checked after every step: the C oracle and the device source compiled
for the CPU (tools/hostsim.cpp, register and generic env views) hold exactly the cumulative
counts the reference printed since the reset."""
import glob
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "env_*.npz")))
IDS = [os.path.basename(f)[4:-4] for f in FILES]


def _golden(path):
    g = np.load(path)
    ev = np.load(path.replace("env_", "events_"))["events"].astype(np.int64)  # [E, T, 5] per step
    return g, np.cumsum(ev, axis=1)


def test_event_fixtures_cover_every_event():
    tot = sum(np.load(f.replace("env_", "events_"))["events"].sum(axis=(0, 1)) for f in FILES)
    assert (tot > 0).all(), tot


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_oracle_events_match_reference_prints(path):
    from oracle import OracleEnv
    g, cum = _golden(path)
    E, T = g["obs"].shape[:2]
    envs = [OracleEnv(str(g["variant"]), int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                      seed=int(g["seed_base"]) + e) for e in range(E)]
    for o in envs:
        o.reset()
        assert not o.events().any()
    for t in range(T):
        for e, o in enumerate(envs):
            o.step(g["actions"][e, t])
            assert np.array_equal(o.events(), cum[e, t]), (e, t)


@pytest.fixture(scope="module")
def hostsim():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools")])
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import hostsim as hs
    return hs


@pytest.mark.parametrize("view", ["default", "generic"])
@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_device_source_events_match_reference_prints(hostsim, path, view):
    g, cum = _golden(path)
    E, T = g["obs"].shape[:2]
    h = hostsim.HostVec(str(g["variant"]), E, int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                        seed_base=int(g["seed_base"]), flags=2 if view == "generic" else 0)
    h.reset()
    assert not h.events().any()
    for t in range(T):
        h.step(g["actions"][:, t])
        assert np.array_equal(h.events(), cum[:, t]), t
    h.reset()  # counters are per episode
    assert not h.events().any()
