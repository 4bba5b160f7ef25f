"""ctypes wrapper of tools/libhostsim.so (device env source compiled for the CPU)."""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mh-ppo_amd"))
from mhppo import _lib  # noqa: E402
from mhppo.env import VARIANTS, CAR_B, PED_B, CROSS_B  # noqa: E402

L = ctypes.CDLL(os.path.join(HERE, "libhostsim.so"))
P = ctypes.c_void_p
L.hs_create.restype = P
L.hs_create.argtypes = [ctypes.POINTER(_lib.EnvCfg)]
for n in ("hs_obs_dim", "hs_state_dim"):
    getattr(L, n).restype = ctypes.c_int
    getattr(L, n).argtypes = [P]
L.hs_reset.argtypes = [P, P]
L.hs_choix.argtypes = [P, P]
L.hs_step.argtypes = [P, P, P, P, P, P]
L.hs_state.argtypes = [P, P]
L.hs_events.argtypes = [P, P]


def _p(a):
    return a.ctypes.data_as(P)


class HostVec:
    def __init__(self, variant, N, nb_car, nb_ped, nb_lines, seed_base=0, flags=0):
        c = _lib.EnvCfg()
        c.variant, c.n_envs, c.nb_car, c.nb_ped, c.nb_lines = VARIANTS[variant], N, nb_car, nb_ped, nb_lines
        c.max_episode, c.sin_model, c.dt = 80, 1, 0.3
        for i, v in enumerate(np.ravel(CAR_B)):
            c.car_b[i] = v
        for i, v in enumerate(np.ravel(PED_B)):
            c.ped_b[i] = v
        c.cross_b[0], c.cross_b[1] = CROSS_B
        c.seed_base = seed_base
        c.flags = flags
        self.c = c
        self.h = L.hs_create(ctypes.byref(c))
        self.N = N
        self.S = 2 * nb_lines if variant == "scalable" else nb_car
        self.obs_dim = L.hs_obs_dim(self.h)
        self.state_dim = L.hs_state_dim(self.h)

    def reset(self):
        o = np.zeros((self.N, self.obs_dim), np.float32)
        L.hs_reset(self.h, _p(o))
        return o

    def choix_test(self):
        o = np.zeros((self.N, self.obs_dim), np.float32)
        assert L.hs_choix(self.h, _p(o)) == 0
        return o

    def step(self, a):
        a = np.ascontiguousarray(a, np.float64)
        o = np.zeros((self.N, self.obs_dim), np.float32)
        r = np.zeros((self.N, self.S)); rl = np.zeros((self.N, self.S)); d = np.zeros(self.N, np.uint8)
        L.hs_step(self.h, _p(a), _p(o), _p(r), _p(rl), _p(d))
        return o, r, rl, d.astype(bool)

    def state(self):
        s = np.zeros((self.N, self.state_dim))
        L.hs_state(self.h, _p(s))
        return s

    def events(self):
        e = np.zeros((self.N, 5), np.uint32)
        L.hs_events(self.h, _p(e))
        return e
