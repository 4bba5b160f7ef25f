"""Quick env-step throughput probe: python tools/bench_env.py variant nb_car nb_ped nb_lines N steps"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo.env import VecCrosswalk  # noqa: E402

v, nc, npd, nl, N, T = sys.argv[1], *map(int, sys.argv[2:7])
env = VecCrosswalk(v, N, nc, npd, nl, seed_base=0)
S = env.n_slots
g = torch.Generator(device="cuda").manual_seed(0)
acts = torch.rand((T, N, 2 * S), device="cuda", dtype=torch.float64, generator=g) * 6 - 4
acts[:, :, S:] = torch.sign(acts[:, :, S:] + 1)
torch.cuda.synchronize()
t0 = time.time(); env.reset(want_obs=False); torch.cuda.synchronize(); tr = time.time() - t0
for want_obs in (False, True):
    env.reset(want_obs=False)
    torch.cuda.synchronize()
    t0 = time.time()
    for t in range(T):
        env.step(acts[t], want_obs=want_obs)
    torch.cuda.synchronize()
    dtm = time.time() - t0
    print(f"{v} N={N} obs={want_obs}: reset {tr*1e3:.2f} ms, {T} steps {dtm*1e3:.2f} ms -> {N*T/dtm/1e6:.2f} M env-steps/s")
