"""Per-step durations of the fused sample+env-step kernel over a rollout (80 steps, 65 536 envs),
from the dispatch-attached HIP events (mhppo_kernel_timing_end_each): which steps make the
spread of the kernel's launch times.  ROLLOUT_CFG="variant nb_car nb_ped nb_lines" (default the
bench's config 3), ITERS iterations after one warm-up; prints one line per step (mean over the
iterations) and a summary.  Usage: python tools/env_steps.py [out.json]"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo import _lib  # noqa: E402
from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

_v, _nc, _np, _nl = (os.environ.get("ROLLOUT_CFG") or "4cars 4 1 2").split()
N = int(os.environ.get("ENVS", 65536))
ITERS = int(os.environ.get("ITERS", 4))
venv = VecCrosswalk(_v, N, int(_nc), int(_np), int(_nl), seed_base=0)
torch.manual_seed(0)
algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
T = 80
L = _lib.lib()
per = []
with torch.no_grad():
    for it in range(ITERS + 1):
        algo.rollout.reset()
        torch.cuda.synchronize()
        _lib.check(L.mhppo_kernel_timing_begin(T))
        algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0,
                                 iteration=it, parts=1, graph=False)
        buf = (ctypes.c_float * T)()
        n = ctypes.c_int32(0)
        _lib.check(L.mhppo_kernel_timing_end_each(buf, T, ctypes.byref(n)))
        assert n.value == T, n.value
        if it:
            per.append([buf[t] * 1e3 for t in range(T)])
mean = [sum(p[t] for p in per) / len(per) for t in range(T)]
for t in range(T):
    print(f"step {t:2d}: {mean[t]:6.1f} us  " + " ".join(f"{p[t]:6.1f}" for p in per), flush=True)
srt = sorted(mean)
print(f"{_v} {_nc}/{_np}/{_nl} N={N}: mean {sum(mean) / T:.1f} us, min {srt[0]:.1f}, median {srt[T // 2]:.1f}, "
      f"max {srt[-1]:.1f}; slowest steps {sorted(range(T), key=lambda t: -mean[t])[:8]}")
if len(sys.argv) > 1:
    json.dump({"cfg": [_v, _nc, _np, _nl], "N": N, "us_per_step": mean, "iters": per}, open(sys.argv[1], "w"))
