"""Generate tests/golden/events_<name>.npz: the reference envs' detection prints counted per
env and step (build container only).

Replays exactly the cases of make_env_golden.py (same per-env streams, same forced actions)
with each env step's stdout captured, and counts the five messages pedestrian.detection prints
("Accident! : ", "Possible accident! ", "Small mistake - priority ? ", "Pedestrian is not
waiting ", "Mauvais signal vert "; Env_hybrid_multi_coop_scalable.py:186,200,222,227,236,
4cars :293-334): events int16 [E, T, 5] = the prints of step t of env e.  The replay's
observations are checked against the committed env_<name>.npz first, so the counts belong to
those fixtures' trajectories.
Run:  python3 tests/golden/gen/make_events_golden.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_env_golden as G  # noqa: E402


def main():
    for name, case in G.CASES.items():
        d = G.run_case(*case, capture_events=True)
        ref = np.load(os.path.join(G.OUT, f"env_{name}.npz"))
        assert np.array_equal(d["obs"], ref["obs"]) and np.array_equal(d["actions"], ref["actions"]), name
        path = os.path.join(G.OUT, f"events_{name}.npz")
        np.savez_compressed(path, events=d["events"])
        print(name, d["events"].sum(axis=(0, 1)), os.path.getsize(path))


if __name__ == "__main__":
    main()
