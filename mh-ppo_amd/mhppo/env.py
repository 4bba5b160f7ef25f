"""Vectorised crosswalk envs on the GPU: N reference envs per handle.

`VecCrosswalk` owns one libmhppo env handle (device state + N CPython-compatible
random streams) and exchanges torch tensors on the handle's device.  It is the
batched form of the reference Gym env
(`Crosswalk_hybrid_multi_*.reset/step`, Environments/Env_hybrid_multi_coop.py
:745-893); `mhppo.envs` wraps it back into the single-env Gym surface.
"""
import ctypes

import torch

from . import _lib

FIX_SCALABLE_LANES = 1  # MHPPO_FIX_SCALABLE_LANES
GENERIC_STEP = 2  # MHPPO_GENERIC_STEP
VARIANTS = {"coop": 0, "4cars": 1, "scalable": 2, "naif": 3, "4cars2": 4, "stop": 5}
CAR_B = ((-4.0, 10.0), (2.0, 10.0))   # Coop-MH-PPO-scalable.py:1007
PED_B = ((-0.05, 0.75, 0.0, -3.0), (0.05, 1.75, 4.0, -0.5))  # :1008
CROSS_B = (2.5, 3.0)  # :1009


def _flat(x, n):
    import numpy as np
    a = np.asarray(x, dtype=np.float64).reshape(-1)
    if a.size != n:
        raise ValueError(f"expected {n} values, got {a.size}")
    return a


# the reference env's detection prints, counted per env (include/mhppo.h MHPPO_EV_*)
EVENT_NAMES = ("Accident! : ", "Possible accident! ", "Small mistake - priority ? ", "Pedestrian is not waiting ",
               "Mauvais signal vert ")


class VecCrosswalk:
    """N independent crosswalk envs of one reference variant on one GPU.

    Env `e` draws from `random.seed(seed_base + env_id_offset + e)`, so a shard
    of envs on rank r reproduces exactly the trajectories the same global env
    ids have on a single GPU.
    """

    def __init__(self, variant, n_envs, nb_car, nb_ped, nb_lines, dt=0.3, max_episode=80,
                 simulation="sin", car_b=CAR_B, ped_b=PED_B, cross_b=CROSS_B, seed_base=0,
                 env_id_offset=0, device=None, fix_scalable_lanes=False, generic_step=False):
        self.variant = variant
        self.device = torch.device(device if device is not None else "cuda")
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", dev_index)
        cfg = _lib.EnvCfg()
        cfg.variant = VARIANTS[variant]
        cfg.n_envs = n_envs
        cfg.nb_car, cfg.nb_ped, cfg.nb_lines = nb_car, nb_ped, nb_lines
        cfg.max_episode = max_episode
        cfg.sin_model = int(simulation == "sin")
        cfg.dt = dt
        for i, v in enumerate(_flat(car_b, 4)):
            cfg.car_b[i] = v
        for i, v in enumerate(_flat(ped_b, 8)):
            cfg.ped_b[i] = v
        for i, v in enumerate(_flat(cross_b, 2)):
            cfg.cross_b[i] = v
        cfg.seed_base = seed_base
        cfg.env_id_offset = env_id_offset
        cfg.flags = FIX_SCALABLE_LANES if fix_scalable_lanes else 0  # opt-in bug fix, SURVEY §8(f)4
        if generic_step:  # run every step on the generic in-HBM env view (tests compare it with the register view)
            cfg.flags |= GENERIC_STEP
        self.cfg = cfg
        self.n_envs, self.nb_car, self.nb_ped, self.nb_lines = n_envs, nb_car, nb_ped, nb_lines
        self.dt, self.max_episode = dt, max_episode
        h = ctypes.c_void_p()
        L = _lib.lib()
        with torch.cuda.device(self.device):
            _lib.check(L.mhppo_env_create(ctypes.byref(cfg), dev_index, ctypes.byref(h)))
        self._h = h
        self.obs_dim = L.mhppo_env_obs_dim(h)
        self.n_slots = L.mhppo_env_slots(h)              # action slots: actions are [N, 2 * n_slots]
        self.n_reward_slots = L.mhppo_env_reward_slots(h)  # reward / reward_light width
        self.state_dim = L.mhppo_env_state_dim(h)

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().mhppo_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _t(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    def reset(self, want_obs=True):
        obs = self._t((self.n_envs, self.obs_dim), torch.float32) if want_obs else None
        _lib.check(_lib.lib().mhppo_env_reset(self._h, _lib.ptr(obs), _lib.stream_ptr(device=self.device)))
        return obs

    def step(self, actions, want_obs=True):
        """actions: float64 [N, 2S] (acc..., light...) on the device."""
        a = actions.to(device=self.device, dtype=torch.float64).contiguous()
        if a.shape != (self.n_envs, 2 * self.n_slots):
            raise ValueError(f"actions must be [{self.n_envs}, {2 * self.n_slots}], got {tuple(a.shape)}")
        obs = self._t((self.n_envs, self.obs_dim), torch.float32) if want_obs else None
        rew = self._t((self.n_envs, self.n_reward_slots), torch.float64)
        rl = self._t((self.n_envs, self.n_reward_slots), torch.float64)
        done = self._t((self.n_envs,), torch.uint8)
        _lib.check(_lib.lib().mhppo_env_step(self._h, _lib.ptr(a), _lib.ptr(obs), _lib.ptr(rew), _lib.ptr(rl),
                                             _lib.ptr(done), _lib.stream_ptr(device=self.device)))
        return obs, rew, rl, done.bool()

    def get_state(self):
        """[N, state_dim] float64: per ped 20, per car slot 8, cross, time, ped_traffic, car_traffic, ped exist."""
        out = self._t((self.n_envs, self.state_dim), torch.float64)
        _lib.check(_lib.lib().mhppo_env_get_state(self._h, _lib.ptr(out), _lib.stream_ptr(device=self.device)))
        return out

    def get_rng(self):
        mt = self._t((self.n_envs, 624), torch.int32)
        mti = self._t((self.n_envs,), torch.int32)
        _lib.check(_lib.lib().mhppo_env_get_rng(self._h, _lib.ptr(mt), _lib.ptr(mti), _lib.stream_ptr(device=self.device)))
        return mt, mti

    def events(self):
        """Event counters, int32 [N, 5] (EVENT_NAMES order): how often each of the
        reference env's detection prints would have fired in every env since its last reset
        (mhppo_env_events; Env_hybrid_multi_coop_scalable.py:186, 200, 222, 227, 236)."""
        out = self._t((self.n_envs, len(EVENT_NAMES)), torch.int32)
        _lib.check(_lib.lib().mhppo_env_events(self._h, _lib.ptr(out), _lib.stream_ptr(device=self.device)))
        return out

    # ------------------------------------------------------------ checkpoint
    def _cfg_key(self):
        c = self.cfg
        return [int(c.variant), int(c.n_envs), int(c.nb_car), int(c.nb_ped), int(c.nb_lines), int(c.max_episode),
                int(c.sin_model), int(c.flags), float(c.dt), [float(x) for x in c.car_b], [float(x) for x in c.ped_b],
                [float(x) for x in c.cross_b], int(c.seed_base), int(c.env_id_offset)]

    # Layout version of the exported device blob (mhppo_env_export): bump whenever the blob's
    # layout changes, even at the same size.  3 = r06 layout (the cars' line / existence bytes,
    # Bufs.carb, between the event counters and the MT blocks); 2 = r03 layout (event counters before
    # the MT blocks, the 4-block MT19937 ring, EI_MTB = active block + stale bits); 1 = r02 (2 MT blocks).
    STATE_LAYOUT = 3

    def state_dict(self):
        """Whole device state (all env fields + every env's MT19937 stream), for exact resume."""
        L = _lib.lib()
        n = int(L.mhppo_env_state_bytes(self._h))
        blob = torch.empty(n, dtype=torch.uint8, device=self.device)
        _lib.check(L.mhppo_env_export(self._h, _lib.ptr(blob), _lib.stream_ptr(device=self.device)))
        return {"cfg": self._cfg_key(), "layout": self.STATE_LAYOUT, "blob": blob.cpu()}

    @staticmethod
    def blob_layout(sd, state_bytes=None):
        """The layout version of an exported blob.  Checkpoints written before the key existed
        (r02 and r03) carry none: an r03 blob is layout 2 and has the layout-2 size (four MT blocks
        per env), an r02 blob is smaller (two), so a key-less blob of the size this build's layout 2
        exports (`state_bytes`) is layout 2 and any other key-less blob layout 1."""
        if "layout" in sd:
            return int(sd["layout"])
        blob = sd.get("blob")
        if blob is not None and state_bytes is not None and int(blob.numel()) == int(state_bytes):
            return 2
        return 1

    def load_state_dict(self, sd):
        n = None if "layout" in sd or self.STATE_LAYOUT != 2 else int(_lib.lib().mhppo_env_state_bytes(self._h))
        lay = VecCrosswalk.blob_layout(sd, n)
        if lay != self.STATE_LAYOUT:
            raise ValueError(f"env checkpoint has state layout {lay}, this build reads layout {self.STATE_LAYOUT} "
                             "(the blob layout changed between versions; it cannot be converted)")
        if list(sd["cfg"]) != self._cfg_key():
            raise ValueError("env checkpoint was made for another configuration")
        L = _lib.lib()
        blob = sd["blob"].to(device=self.device, dtype=torch.uint8).contiguous()
        if blob.numel() != int(L.mhppo_env_state_bytes(self._h)):
            raise ValueError("env checkpoint size mismatch")
        _lib.check(L.mhppo_env_import(self._h, _lib.ptr(blob), _lib.stream_ptr(device=self.device)))
        torch.cuda.current_stream(self.device).synchronize()

    def device_scope(self):
        """Context making the handle's device current (torch allocations and the ppo kernels,
        which take no handle, then run on it)."""
        return torch.cuda.device(self.device)
