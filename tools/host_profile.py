"""Host-side cost of one product training iteration (Algo_PPO.train(1)) on a bench config:
cProfile of K iterations (tottime / cumtime tables), plus the wall time of the host's issue of
one iteration against the synchronised iteration time.  A small-N config (2: 4 096 envs) whose
GPU work per launch is short is bound by this host time.
Usage: python tools/host_profile.py [config] [iterations]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
import torch  # noqa: E402

from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

CONFIGS = {3: ("4cars", 4, 1, 2, 65536), 4: ("scalable", 8, 1, 4, 65536), 2: ("coop", 2, 1, 2, 4096)}
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
v, nc, npd, nl, N = CONFIGS[cfg]
venv = VecCrosswalk(v, N, nc, npd, nl, seed_base=0, device="cuda:0")
torch.manual_seed(0)
algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0, save_curves=False)
for _ in range(3):
    algo.train(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    algo.train(1)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"config {cfg}: host issue {1e3 * (t1 - t0) / K:.3f} ms/iteration, synchronised {1e3 * (t2 - t0) / K:.3f} ms",
      flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(K):
    algo.train(1)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumtime").print_stats(40)
