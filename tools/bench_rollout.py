"""Rollout collect timing (80 steps of policy + env kernels, 65536 envs; ROLLOUT_CFG selects the
shape, default 4cars 4/1/2), HIP events per kernel."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

# ROLLOUT_CFG="variant nb_car nb_ped nb_lines" (default: the bench's config 3)
_v, _nc, _np, _nl = (os.environ.get("ROLLOUT_CFG") or "4cars 4 1 2").split()
venv = VecCrosswalk(_v, int(os.environ.get("ROLLOUT_N", "65536")), int(_nc), int(_np), int(_nl), seed_base=0)
torch.manual_seed(0)
algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
T = 80
with torch.no_grad():
    for it in range(3):
        ev = [[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(T)]
        r0 = torch.cuda.Event(enable_timing=True); r1 = torch.cuda.Event(enable_timing=True)
        r0.record()
        algo.rollout.reset()
        r1.record()
        a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
        a.record()
        algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0,
                                 iteration=it, step_events=ev)
        b.record()
        torch.cuda.synchronize()
        env_us = sum(e0.elapsed_time(e1) for e0, e1 in ev) / T * 1e3
        g = algo.rollout.gpu
        R = g.rows.numel() - 2 - 2 * (g.parts + 1)
        nc, nw = (int(v) for v in g.rows[R:R + 2].tolist())
        print(f"iter {it}: reset {r0.elapsed_time(r1) * 1e3:.0f} us, collect {a.elapsed_time(b):.2f} ms, "
              f"env kernel {env_us:.1f} us/step; policy rows "
              f"{nc} cross + {nw} wait of {R}", flush=True)
