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
    waves = buf[15]
    tot = sum(buf[k] for k in PHASES)
    print(f"{v} {nc}/{npd}/{nl} N={N}: {waves} wave-launches, collect {ev[0].elapsed_time(ev[1]):.2f} ms")
    for k, name in PHASES.items():
        print(f"  {k:2d} {name:24s} {buf[k] / max(waves, 1):10.0f} cycles/wave  {100.0 * buf[k] / max(tot, 1):5.1f} %")
    print(f"     {'total':24s} {tot / max(waves, 1):10.0f} cycles/wave")


if __name__ == "__main__":
    main()
