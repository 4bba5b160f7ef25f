"""Reference harness — fixture generation in the BUILD container only.

Imports the reference environments from /root/reference under the offline gym
stub (tests/golden/gen/gymstub) and gives each env its own CPython `random`
stream by swapping `random.getstate()/setstate()` around every reset/step
(SURVEY Appendix C.3).  Nothing here is imported by tests, bench or smoke: the
reference never travels to the GPU box, only the .npz fixtures it produced.
"""
import contextlib
import io
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "gymstub"))
sys.path.insert(1, REF)
sys.dont_write_bytecode = True

import numpy as np  # noqa: E402
import gym  # noqa: E402  (the stub)
import Environments  # noqa: E402,F401  (registers the 6 ids)

CAR_B = np.array([[-4.0, 10.], [2.0, 10.]])
PED_B = np.array([[-0.05, 0.75, 0.0, -3.0], [0.05, 1.75, 4., -0.5]])
CROSS_B = np.array([2.5, 3.0])

IDS = {
    "coop": "Crosswalk_hybrid_multi_coop-v0",
    "4cars": "Crosswalk_hybrid_multi_coop_4cars-v0",
    "scalable": "Crosswalk_hybrid_multi_coop_scalable-v0",
    "naif": "Crosswalk_hybrid_multi_naif-v0",
    "4cars2": "Crosswalk_hybrid_multi_coop_4cars2-v0",
    "stop": "Crosswalk_hybrid_multi_stop-v0",
}


def make(variant, nb_car, nb_ped, nb_lines, dt=0.3, max_episode=80, simulation="sin"):
    with contextlib.redirect_stdout(io.StringIO()):
        return gym.make(IDS[variant], car_b=CAR_B, ped_b=PED_B, cross_b=CROSS_B, nb_car=nb_car,
                        nb_ped=nb_ped, nb_lines=nb_lines, dt=dt, max_episode=max_episode,
                        simulation=simulation)


class Stream:
    """One env's private CPython random stream (random.seed(seed))."""

    def __init__(self, seed):
        saved = random.getstate()
        random.seed(seed)
        self.state = random.getstate()
        random.setstate(saved)

    @contextlib.contextmanager
    def active(self):
        saved = random.getstate()
        random.setstate(self.state)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                yield
        finally:
            self.state = random.getstate()
            random.setstate(saved)

    @property
    def mti(self):
        return self.state[1][-1]


def flat(state):
    return np.concatenate([v.flatten() for v in state.values()]).astype(np.float32)


def dump(env):
    out = []
    for d in env.pedestrian:
        out += [d.Sp_x, d.Sp_y, d.Vp_x, d.Vp_y, d.decision, d.at_crossing, d.ped_left, d.ped_in_cross,
                d.accident, d.time_stop, d.stop, d.line_pos, d.waiting_time, d.crossing_time, d.worst_dl,
                d.delta, d.t0, getattr(d, "need_to_stop", 0), d.direction, d.follow_rule]
    for c in env.cars:
        out += [c.Ac, c.Vc, c.Sc, c.light, c.possible_accident, c.error_scenario, c.Ts,
                getattr(c, "exist", True)]
    return np.array(out, dtype=np.float64)
