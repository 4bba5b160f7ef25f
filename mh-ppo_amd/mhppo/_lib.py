"""ctypes binding of libmhppo.so (include/mhppo.h).

The HIP library is the product path: there is no CPU or PyTorch fallback.  If
the shared object is missing or fails to load, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# MHPPO_LIB points at an alternative build of the same library (A/B kernel experiments,
# tools/ab_build.sh); the default is the in-tree build.
LIB_PATH = os.environ.get("MHPPO_LIB") or os.path.join(HERE, "lib", "libmhppo.so")

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
U64 = ctypes.c_uint64
F64 = ctypes.c_double


class EnvCfg(ctypes.Structure):
    _fields_ = [
        ("variant", I32), ("n_envs", I32), ("nb_car", I32), ("nb_ped", I32), ("nb_lines", I32),
        ("max_episode", I32), ("sin_model", I32), ("flags", I32), ("dt", F64),
        ("car_b", F64 * 4), ("ped_b", F64 * 8), ("cross_b", F64 * 2), ("seed_base", U64),
        ("env_id_offset", U64),
    ]


class Mlp(ctypes.Structure):
    _fields_ = [("packed", P), ("n_in", I32), ("n_out", I32), ("kind", I32), ("reserved", I32),
                ("mean", ctypes.c_float), ("std", ctypes.c_float)]


class BucketDst(ctypes.Structure):  # mhppo_bucket_dst
    _fields_ = [("obs", P), ("act", P), ("logp", P), ("ret", P), ("rew", P)]


class RolloutBufs(ctypes.Structure):
    _fields_ = [("feat_d", P), ("probs_d", P), ("logp_d", P), ("a_d", P), ("closest", P),
                ("feat_c", P), ("out_c", P), ("obs", P), ("obs_c", P), ("act", P), ("logp", P),
                ("rew", P), ("ep_min", P), ("exist", P), ("rows", P), ("T", I32),
                ("flags", I32), ("status", P), ("parts", I32), ("reserved", I32), ("rec_of", P)]


class EvalBufs(ctypes.Structure):
    _fields_ = [("obs", P), ("a_d", P), ("trig", P), ("ep_min", P), ("obs_hist", P), ("acts", P), ("rews_c", P),
                ("rews_d", P), ("waiting", P), ("saved", P), ("T", I32), ("reserved", I32)]


# name: (restype, argtypes)
_SIGS = {
    "mhppo_env_create": (I32, [ctypes.POINTER(EnvCfg), I32, ctypes.POINTER(P)]),
    "mhppo_env_destroy": (None, [P]),
    "mhppo_env_obs_dim": (I32, [P]),
    "mhppo_env_slots": (I32, [P]),
    "mhppo_env_reward_slots": (I32, [P]),
    "mhppo_env_state_dim": (I32, [P]),
    "mhppo_env_reset": (I32, [P, P, P]),
    "mhppo_env_choix_test": (I32, [P, P, P]),
    "mhppo_env_state_bytes": (I64, [P]),
    "mhppo_env_export": (I32, [P, P, P]),
    "mhppo_env_import": (I32, [P, P, P]),
    "mhppo_env_step": (I32, [P, P, P, P, P, P, P]),
    "mhppo_env_get_state": (I32, [P, P, P]),
    "mhppo_env_get_rng": (I32, [P, P, P, P]),
    "mhppo_env_events": (I32, [P, P, P]),
    "mhppo_choice_dim": (I32, [P]),
    "mhppo_rollout_begin": (I32, [P, ctypes.POINTER(Mlp), P, P, ctypes.POINTER(RolloutBufs), P]),
    "mhppo_rollout_step": (I32, [P, ctypes.POINTER(Mlp), ctypes.POINTER(Mlp), P, I32,
                                 ctypes.POINTER(RolloutBufs), P]),
    "mhppo_rollout_policy": (I32, [P, ctypes.POINTER(Mlp), ctypes.POINTER(Mlp), ctypes.POINTER(RolloutBufs), P]),
    "mhppo_rollout_sample_env": (I32, [P, P, I32, ctypes.POINTER(RolloutBufs), P]),
    "mhppo_rollout_policy_part": (I32, [P, ctypes.POINTER(Mlp), ctypes.POINTER(Mlp), ctypes.POINTER(RolloutBufs), I32,
                                        P]),
    "mhppo_rollout_sample_env_part": (I32, [P, P, I32, ctypes.POINTER(RolloutBufs), I32, P]),
    "mhppo_kernel_timing_begin": (I32, [I32]),
    "mhppo_kernel_timing_end": (I32, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(I32)]),
    "mhppo_kernel_timing_end_each": (I32, [P, I32, ctypes.POINTER(I32)]),
    "mhppo_eval_step": (I32, [P, ctypes.POINTER(Mlp), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp), I32,
                              ctypes.POINTER(EvalBufs), P]),
    "mhppo_rollout_check": (I32, [ctypes.POINTER(RolloutBufs), P]),
    "mhppo_philox_normal": (I32, [U64, U64, P, I64, P]),
    "mhppo_philox_uniform": (I32, [U64, U64, P, I64, P]),
    "mhppo_philox_normal_2d": (I32, [U64, U64, U64, P, I64, I64, P]),
    "mhppo_libm_eval": (I32, [I32, U64, I64, P, P]),
    "mhppo_returns_scan": (I32, [P, P, I64, I32, F64, P]),
    "mhppo_returns_scan_tm": (I32, [P, P, I64, I32, F64, P]),
    "mhppo_bucket_scatter": (I32, [P, P, I64, I32] + [P] * 7),
    "mhppo_adv_stats": (I32, [P, P, I64, P, P]),
    "mhppo_adv_normalize": (I32, [P, P, I64, P, F64, P, P]),
    "mhppo_ppo_cont_fwd_bwd": (I32, [P, P, P, P, I64, F64, P, P, P]),
    "mhppo_ppo_choice_fwd_bwd": (I32, [P, P, P, I64, P, F64, P, P, P]),
    "mhppo_mse_fwd_bwd": (I32, [P, P, I64, F64, P, P, P]),
    "mhppo_mlp_train": (I32, [I32, I32, P, P, I64, P, P, P, P, P, P, F64, ctypes.c_float, ctypes.c_float, P, P, P]),
    "mhppo_mlp_train_pair": (I32, [P, P, P, I64, P, P, P, P, P, F64, ctypes.c_float, ctypes.c_float, P, P, P, P, P]),
    "mhppo_last_error": (ctypes.c_char_p, []),
    "mhppo_version": (ctypes.c_char_p, []),
}

_lib = None


class MhppoError(RuntimeError):
    pass


class MhppoNaNError(MhppoError, ValueError):
    """MHPPO_ENAN: a NaN policy output was sampled (the reference raises ValueError there)."""

ENAN = -4


def lib():
    """Load libmhppo.so once; raise loudly if it is absent (no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MhppoError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def declared_symbols():
    return list(_SIGS)


def check(rc):
    if rc != 0:
        cls = MhppoNaNError if rc == ENAN else MhppoError
        raise cls(f"libmhppo error {rc}: {lib().mhppo_last_error().decode()}")
    return rc


def ptr(t):
    """Device (or host) pointer of a torch tensor / None."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None, device=None):
    """hipStream_t of `stream`, else of the current stream of `device` (default: the
    current device).  Handle-bound calls pass their handle's device: the library makes
    that device current for the call (include/mhppo.h), so the stream must live there."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)
