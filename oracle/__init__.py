"""ORACLE — test infrastructure only.

ctypes view of oracle/liboracle.so (the C restatement of the reference envs,
CPython random and PPO math).  Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg; the product package (mh-ppo_amd/) never imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
VARIANTS = {"coop": 0, "4cars": 1, "scalable": 2, "naif": 3}
CAR_B = np.array([[-4.0, 10.], [2.0, 10.]])
PED_B = np.array([[-0.05, 0.75, 0.0, -3.0], [0.05, 1.75, 4., -0.5]])
CROSS_B = np.array([2.5, 3.0])

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I, D, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_uint64
        L.oracle_env_create.restype = P
        L.oracle_env_create.argtypes = [I, I, I, I, D, I, I, P, P, P]
        L.oracle_env_destroy.argtypes = [P]
        L.oracle_env_seed.argtypes = [P, U64]
        L.oracle_env_rng_words.restype = U64
        L.oracle_env_rng_words.argtypes = [P]
        L.oracle_env_get_rng.argtypes = [P, P, P]
        L.oracle_env_obs_dim.restype = I
        L.oracle_env_obs_dim.argtypes = [P]
        L.oracle_env_reset.argtypes = [P, P]
        L.oracle_env_step.restype = I
        L.oracle_env_step.argtypes = [P, P, P, P, P]
        L.oracle_env_dump.restype = I
        L.oracle_env_dump.argtypes = [P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """One reference env on its own CPython random stream."""

    def __init__(self, variant, nb_car, nb_ped, nb_lines, dt=0.3, max_episode=80, sin=True, seed=None):
        L = lib()
        self.variant = variant
        self.nb_car, self.nb_ped, self.nb_lines = nb_car, nb_ped, nb_lines
        self.S = 2 * nb_lines if variant == "scalable" else nb_car
        self._cb = np.ascontiguousarray(CAR_B, dtype=np.float64)
        self._pb = np.ascontiguousarray(PED_B, dtype=np.float64)
        self._xb = np.ascontiguousarray(CROSS_B, dtype=np.float64)
        self.h = L.oracle_env_create(VARIANTS[variant], nb_car, nb_ped, nb_lines, dt, max_episode, int(sin),
                                     _p(self._cb), _p(self._pb), _p(self._xb))
        if not self.h:
            raise ValueError("oracle_env_create rejected the shape")
        self.obs_dim = L.oracle_env_obs_dim(self.h)
        if seed is not None:
            L.oracle_env_seed(self.h, seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_env_destroy(self.h)
            self.h = None

    def reset(self):
        o = np.zeros(self.obs_dim, np.float32)
        lib().oracle_env_reset(self.h, _p(o))
        return o

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.float64)
        o = np.zeros(self.obs_dim, np.float32)
        r = np.zeros(self.S, np.float64)
        rl = np.zeros(self.S, np.float64)
        d = lib().oracle_env_step(self.h, _p(a), _p(o), _p(r), _p(rl))
        return o, r, rl, bool(d)

    def dump(self):
        out = np.zeros(20 * self.nb_ped + 8 * self.S, np.float64)
        n = lib().oracle_env_dump(self.h, _p(out))
        return out[:n]

    @property
    def rng_words(self):
        return lib().oracle_env_rng_words(self.h)

    def rng_state(self):
        mt = np.zeros(624, np.uint32)
        mti = np.zeros(1, np.int32)
        lib().oracle_env_get_rng(self.h, _p(mt), _p(mti))
        return mt, int(mti[0])


def rng_stream(seed, kind, n, a=0.0, b=0.0, per=1):
    L = lib()
    L.oracle_rng_stream.restype = ctypes.c_int
    L.oracle_rng_stream.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_int, ctypes.c_void_p]
    out = np.zeros(n * per, np.float64)
    k = L.oracle_rng_stream(seed, kind, a, b, n, _p(out))
    return out[:k]
