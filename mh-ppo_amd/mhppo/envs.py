"""Gym-compatible single-env surface of the reference environments.

Replaces `gym.make("Crosswalk_hybrid_multi_*-v0", car_b=..., ped_b=..., cross_b=...,
nb_car=..., nb_ped=..., nb_lines=..., dt=..., max_episode=..., simulation=...)`
(Environments/__init__.py:3-42; Coop-MH-PPO-scalable.py:1027) with the same
constructor keywords and the surface the reference drivers touch:
  reset(seed=None, options=None) -> (OrderedDict car|car_follow|env|ped float32, {})
  step(actions float64[2S])      -> (state, rewards float64[S], done, False, {})
  observation_space["car"|"env"|"ped"].shape, action_space.shape, reward_light,
  cars[i].exist / .Sc / .Vc ..., pedestrian[j].waiting_time ..., nb_car, nb_ped,
  nb_lines, car_b, dt, speed_limit, max_episode, cross, ped_traffic, car_traffic,
  get_state().
The backend is a 1-env VecCrosswalk on the GPU (the product path).  Like the
reference module (`random.seed(10)` at import, Env_hybrid_multi_coop.py:10), a
fresh env draws from random.seed(10); `seed=` picks another stream.  As in the
reference, reset's `seed` only reseeds an unused numpy generator.
"""
from collections import OrderedDict

import numpy as np

VARIANT_OF_ID = {
    "Crosswalk_hybrid_multi_coop-v0": "coop",
    "Crosswalk_hybrid_multi_coop_4cars-v0": "4cars",
    "Crosswalk_hybrid_multi_coop_scalable-v0": "scalable",
    "Crosswalk_hybrid_multi_naif-v0": "naif",
    "Crosswalk_hybrid_multi_coop_4cars2-v0": "4cars2",
    "Crosswalk_hybrid_multi_stop-v0": "stop",
}
_REGISTRY = {}


class Box:
    def __init__(self, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = dtype

    def sample(self):
        return np.zeros(self.shape, self.dtype)


class Dict:
    def __init__(self, spaces):
        self.spaces = OrderedDict(sorted(spaces.items()))  # gym 0.26 sorts plain-dict keys

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()


class _View:
    """Attribute view of one car / pedestrian, read from the backend's state vector."""

    def __init__(self, fields):
        self.__dict__.update(fields)


PED_FIELDS = ("Sp_x", "Sp_y", "Vp_x", "Vp_y", "decision", "at_crossing", "ped_left", "ped_in_cross", "accident",
              "time_stop", "stop", "line_pos", "waiting_time", "crossing_time", "worst_dl", "delta", "t0",
              "need_to_stop", "direction", "follow_rule")
CAR_FIELDS = ("Ac", "Vc", "Sc", "light", "possible_accident", "error_scenario", "Ts", "exist")


class CrosswalkEnv:
    def __init__(self, car_b, ped_b, cross_b, nb_car, nb_ped, nb_lines, dt, max_episode, simulation="unif",
                 variant="coop", seed=10, device=None, backend=None):
        self.variant = variant
        self.car_b, self.ped_b, self.cross_b = np.asarray(car_b), np.asarray(ped_b), np.asarray(cross_b)
        self.nb_car, self.nb_ped, self.nb_lines = nb_car, nb_ped, nb_lines
        self.dt, self.max_episode, self.simulation = dt, max_episode, simulation
        self.speed_limit = 10
        self.Vm, self.tau, self.car_size = 2.5, 1.0, 4.0
        self.S = 2 * nb_lines if variant == "scalable" else nb_car  # AV slots (rewards, cars[])
        self.nA = 2 * nb_car if variant == "4cars2" else self.S     # action slots (4cars2: + followers)
        self.nC = 2 * nb_car if variant in ("4cars", "4cars2") else self.S
        cw = 7 if variant == "scalable" else 6
        spaces = {"car": Box((self.S * cw,)), "env": Box((4 if variant == "scalable" else 3,)),
                  "ped": Box((nb_ped * 9,))}
        if variant in ("4cars", "4cars2"):
            spaces["car_follow"] = Box((nb_car * 6,))
        self.observation_space = Dict(spaces)
        self.action_space = Box((2 * self.nA,))
        self._seed, self._device, self._backend = seed, device, backend
        self.reward_light = 0.0
        self.state = None

    # ----------------------------------------------------------------- backend
    @property
    def venv(self):
        if self._backend is None:
            from .env import VecCrosswalk
            self._backend = VecCrosswalk(self.variant, 1, self.nb_car, self.nb_ped, self.nb_lines, dt=self.dt,
                                         max_episode=self.max_episode, simulation=self.simulation,
                                         car_b=self.car_b, ped_b=self.ped_b, cross_b=self.cross_b,
                                         seed_base=self._seed, device=self._device)
        return self._backend

    def _np(self, x):
        return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)

    def _split(self, flat):
        out, k = OrderedDict(), 0
        for name, sp in self.observation_space.spaces.items():
            n = sp.shape[0]
            out[name] = flat[k:k + n].astype(np.float32)
            k += n
        return out

    def _refresh(self):
        st = self._np(self.venv.get_state())[0]
        P = self.nb_ped
        self.pedestrian = [_View(dict(zip(PED_FIELDS, st[20 * p:20 * p + 20]))) for p in range(P)]
        tail = 20 * P + 8 * self.nC
        for j, p in enumerate(self.pedestrian):
            p.exist = bool(st[tail + 4 + j])
        base = 20 * P
        self.cars = [_View(dict(zip(CAR_FIELDS, st[base + 8 * i:base + 8 * i + 8]))) for i in range(self.S)]
        for c in self.cars:
            c.exist = bool(c.exist)
        fb = base + 8 * self.S
        self.cars_follow = [_View(dict(zip(CAR_FIELDS, st[fb + 8 * i:fb + 8 * i + 8])))
                            for i in range(self.nC - self.S)]
        self.cross, self.time = st[tail], st[tail + 1]
        self.ped_traffic, self.car_traffic = int(st[tail + 2]), int(st[tail + 3])

    # ------------------------------------------------------------------ gym API
    def seed(self, seed=None):
        self.np_rand = np.random.default_rng(seed)
        return [seed]

    def reset(self, seed=None, options=None):
        if seed is not None:
            self.seed(seed)
        obs = self._np(self.venv.reset())[0]
        self.state = self._split(obs)
        self.reward_light = 0.0
        self._refresh()
        return self.state, {}

    def step(self, actions):
        import torch
        a = np.asarray(actions, dtype=np.float64).reshape(1, -1)
        if a.shape[1] != 2 * self.nA:
            raise ValueError(f"expected {2 * self.nA} actions, got {a.shape[1]}")
        ta = torch.from_numpy(a)
        if hasattr(self.venv, "device"):
            ta = ta.to(self.venv.device)
        obs, rew, rl, done = self.venv.step(ta)
        self.state = self._split(self._np(obs)[0])
        self.reward_light = self._np(rl)[0].astype(np.float64)
        self._refresh()
        return self.state, self._np(rew)[0].astype(np.float64), bool(self._np(done)[0]), False, {}

    def get_state(self):
        return self.state

    def close(self):
        pass


def register(id, entry_point=None, max_episode_steps=None, reward_threshold=None, **kwargs):
    _REGISTRY[id] = VARIANT_OF_ID.get(id, kwargs.get("variant"))


def make(id, **kwargs):
    """gym.make replacement for the four reference ids (Environments/__init__.py)."""
    variant = _REGISTRY.get(id) or VARIANT_OF_ID.get(id)
    if variant is None:
        raise KeyError(f"unknown env id {id!r}; known: {sorted(VARIANT_OF_ID)}")
    return CrosswalkEnv(variant=variant, **kwargs)


for _id in VARIANT_OF_ID:
    register(_id)
