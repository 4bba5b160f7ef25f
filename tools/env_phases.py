"""Per-phase cycle breakdown of the fused sample+env-step kernel (k_sample_env_r) from a
timing build:  tools/ab_build.sh timing -DMHPPO_TIMING
               MHPPO_LIB=build_ab/timing/libmhppo.so python tools/env_phases.py [variant nc np nl N]
Prints mean shader-clock cycles per wave and launch for each phase (lane-0 view)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo import _lib  # noqa: E402
from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

PHASES = {1: "MT refill (wave)", 2: "env state load (EnvR)", 3: "select + MVN action", 4: "car steps (+IDM)",
          5: "pedestrian step", 6: "detection", 7: "rewards", 11: "observe: car rows",
          12: "observe: ped get_data", 8: "observe: obs block store", 9: "commit", 10: "rollout buffer writes"}


def per_step(algo, fn, buf):
    fmax = _lib.lib().mhppo_debug_timing_max
    fmax.restype, fmax.argtypes = ctypes.c_int32, [ctypes.c_void_p]
    bmax = (ctypes.c_uint64 * 16)()
    """Phase cycles per wave of every step of one rollout (the collect loop of RolloutGPU.collect,
    synchronised and read back after each env-step launch)."""
    L = _lib.lib()
    ro = algo.rollout.gpu
    algo.rollout.reset()
    with torch.no_grad():
        ro.draw_noise(0, 2)
        mc, tc = algo.actor_net_choice.mlp_desc()
        mx, tx = algo.actor_net_cross.mlp_desc()
        mw, tw = algo.actor_net_wait.mlp_desc()
        st = _lib.stream_ptr()
        _lib.check(L.mhppo_rollout_begin(ro.venv.handle, ctypes.byref(mc), _lib.ptr(ro.u), None, ctypes.byref(ro._bufs),
                                         st))
        rows = []
        for t in range(ro.T):
            if ro.P == 1:
                ro._bufs.feat_c = ro.obs_c[t].data_ptr()
            _lib.check(L.mhppo_rollout_policy(ro.venv.handle, ctypes.byref(mx), ctypes.byref(mw),
                                              ctypes.byref(ro._bufs), st))
            torch.cuda.synchronize()
            fn(buf)  # clears
            _lib.check(L.mhppo_rollout_sample_env(ro.venv.handle, _lib.ptr(ro.eps[t]), t, ctypes.byref(ro._bufs), st))
            torch.cuda.synchronize()
            fmax(bmax)
            fn(buf)
            w = max(buf[15], 1)
            rows.append(([buf[k] / w for k in PHASES], buf[14], [bmax[k] for k in PHASES]))
    print("step " + " ".join(f"{PHASES[k][:10]:>10s}" for k in PHASES) + "  (mean wave / slowest wave per phase)")
    for t, (r, mx, pm) in enumerate(rows):
        print(f"{t:4d} " + " ".join(f"{x:10.0f}" for x in r) + f"  total {sum(r):8.0f}  max {mx:8d}")
        print("  max" + " ".join(f"{x:10d}" for x in pm))


def main():
    v, nc, npd, nl, N = (sys.argv[1:2] or ["4cars"])[0], *map(int, (sys.argv[2:6] or [4, 1, 2, 65536]))
    venv = VecCrosswalk(v, N, nc, npd, nl, seed_base=0)
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
    L = _lib.lib()
    fn = L.mhppo_debug_timing
    fn.restype, fn.argtypes = ctypes.c_int32, [ctypes.c_void_p]
    buf = (ctypes.c_uint64 * 16)()
    with torch.no_grad():
        algo.rollout.reset()
        algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0, iteration=0)
        torch.cuda.synchronize()
        fn(buf)  # discard the warm-up iteration
        algo.rollout.reset()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0, iteration=1)
        ev[1].record()
        torch.cuda.synchronize()
        fn(buf)
    if os.environ.get("PER_STEP"):  # one more iteration, phases read back after every step
        per_step(algo, fn, buf)
    waves = buf[15]
    tot = sum(buf[k] for k in PHASES)
    print(f"{v} {nc}/{npd}/{nl} N={N}: {waves} wave-launches, collect {ev[0].elapsed_time(ev[1]):.2f} ms")
    for k, name in PHASES.items():
        print(f"  {k:2d} {name:24s} {buf[k] / max(waves, 1):10.0f} cycles/wave  {100.0 * buf[k] / max(tot, 1):5.1f} %")
    print(f"     {'total':24s} {tot / max(waves, 1):10.0f} cycles/wave")


if __name__ == "__main__":
    main()
