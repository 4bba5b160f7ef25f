"""Diagnostic: Algo_PPO.train(1) with the pipelined epochs (pairs on / off) vs ten ppo.train_epoch
calls; prints which nets differ and by how much (max |diff|)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
import torch  # noqa: E402

from mhppo import ppo  # noqa: E402
from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

pipelined = ppo.train_epochs


def sequential(heads, n_epochs, bucket=None):
    out = None
    for _ in range(n_epochs):
        out = ppo.train_epoch(heads, bucket)
    return out


N = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
ITERS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
res = {}
for arm in ("pairs", "no_pairs", "train_epoch"):
    ppo.PIPELINE_PAIRS = arm == "pairs"
    ppo.train_epochs = sequential if arm == "train_epoch" else pipelined
    venv = VecCrosswalk("4cars", N, 4, 1, 2, seed_base=5)
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=1, save_curves=False)
    res[arm] = []
    for it in range(ITERS):
        algo.train(1)
        res[arm].append([n.flat().detach().cpu().clone() for n in algo.nets()])
names = ["actor_cross", "actor_wait", "actor_choice", "critic_cross", "critic_wait", "critic_choice"]
for it in range(ITERS):
    for a, b in (("pairs", "train_epoch"), ("no_pairs", "train_epoch"), ("pairs", "no_pairs")):
        print("iteration", it + 1, a, "vs", b,
              [(nm, float((x - y).abs().max())) for nm, x, y in zip(names, res[a][it], res[b][it])])
