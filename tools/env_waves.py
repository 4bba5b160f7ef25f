"""Per-wave durations of the fused sample+env-step kernel, step by step, from an A/B build that
stamps each wave's shader clock at its start and end (tools/ab_build.sh waves -DMHPPO_WAVE_TIMES;
MHPPO_LIB=build_ab/waves/libmhppo.so python tools/env_waves.py [variant nc np nl N]).  A launch
lasts as long as its slowest wave (one wave per SIMD at 65 536 envs): this shows how the wave
durations of each step are spread.  Prints per step: mean / median / p90 / max wave cycles and
the launch span (last end - first start)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo import _lib  # noqa: E402
from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402


def main():
    v, nc, npd, nl, N = (sys.argv[1:2] or ["4cars"])[0], *map(int, (sys.argv[2:6] or [4, 1, 2, 65536]))
    venv = VecCrosswalk(v, N, nc, npd, nl, seed_base=0)
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
    L = _lib.lib()
    fn = L.mhppo_debug_wave_times
    fn.restype, fn.argtypes = ctypes.c_int32, [ctypes.c_void_p]
    buf = (ctypes.c_uint64 * (2 * 8192))()
    ro = algo.rollout.gpu
    W = (N + 63) // 64
    with torch.no_grad():
        ro.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0, iteration=0)  # warm-up
        algo.rollout.reset()
        ro.draw_noise(0, 1)
        mc, tc = algo.actor_net_choice.mlp_desc()
        mx, tx = algo.actor_net_cross.mlp_desc()
        mw, tw = algo.actor_net_wait.mlp_desc()
        st = _lib.stream_ptr()
        _lib.check(L.mhppo_rollout_begin(ro.venv.handle, ctypes.byref(mc), _lib.ptr(ro.u), None, ctypes.byref(ro._bufs),
                                         st))
        print("step   mean  median    p90    max   span  (shader cycles per wave)")
        allw = []
        for t in range(ro.T):
            if ro.P == 1:
                ro._bufs.feat_c = ro.obs_c[t].data_ptr()
            _lib.check(L.mhppo_rollout_policy(ro.venv.handle, ctypes.byref(mx), ctypes.byref(mw),
                                              ctypes.byref(ro._bufs), st))
            _lib.check(L.mhppo_rollout_sample_env(ro.venv.handle, _lib.ptr(ro.eps[t]), t, ctypes.byref(ro._bufs), st))
            fn(buf)
            a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 2)[:W].astype(np.int64)
            d = a[:, 1] - a[:, 0]
            allw.append(d)
            print(f"{t:4d} {d.mean():7.0f} {np.median(d):7.0f} {np.percentile(d, 90):6.0f} {d.max():6d} "
                  f"{a[:, 1].max() - a[:, 0].min():6d}", flush=True)
        allw = np.stack(allw)  # [T, W]
        slow = allw.argmax(1)
        print(f"slowest wave per step (wave index = env // 64): {slow.tolist()}")
        rank = allw.mean(0).argsort()[::-1][:10]
        print(f"waves slowest on average: {rank.tolist()} ({allw.mean(0)[rank].round().tolist()} cycles; "
              f"all-wave mean {allw.mean():.0f})")


if __name__ == "__main__":
    main()
