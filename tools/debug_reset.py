"""Debug: GPU env reset vs the C oracle for one shape (mismatching envs, the first differing obs
fields, RNG cursors).  usage: python tools/debug_reset.py variant nb_car nb_ped nb_lines [N] [resets]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo.env import VecCrosswalk  # noqa: E402
from oracle import OracleBatch  # noqa: E402

v, nc, npd, nl = sys.argv[1], *map(int, sys.argv[2:5])
N = int(sys.argv[5]) if len(sys.argv) > 5 else 512
K = int(sys.argv[6]) if len(sys.argv) > 6 else 1
env = VecCrosswalk(v, N, nc, npd, nl, seed_base=9000)
orc = OracleBatch(v, N, nc, npd, nl, seed_base=9000)
for k in range(K):
    g = env.reset().cpu().numpy()
    o = orc.reset()
    bad = np.nonzero((g != o).any(1))[0]
    mt_g, mti_g = env.get_rng()
    mt_o, mti_o = orc.rng_state()
    mti_g = mti_g.cpu().numpy()
    print(f"reset {k}: {len(bad)} of {N} envs differ; RNG cursor differs in {int((mti_g != mti_o).sum())} envs")
    for e in bad[:5]:
        f = np.nonzero(g[e] != o[e])[0]
        print(f"  env {e}: fields {f[:12].tolist()} gpu {g[e][f[:4]].tolist()} oracle {o[e][f[:4]].tolist()} "
              f"mti gpu {int(mti_g[e])} oracle {int(mti_o[e])}")
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    env.reset(want_obs=False)
e1.record()
torch.cuda.synchronize()
print(f"reset time {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per reset ({N} envs)")
