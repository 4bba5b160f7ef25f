"""One PPO iteration (rollout + update) on this rank's shard of `--envs-total` envs, then
rank 0 saves every net's flat parameters (tests/test_dp_gpu.py; run under torchrun or alone).
The envs shard by global id (env_id_offset), as bench.py / DESIGN.md §6.
--nccl-world1: one rank on RCCL (backend "nccl", bound to the GPU as bench.py binds it) with
the data-parallel collectives forced on, so every all-reduce of the update runs through RCCL
on a one-GPU box (a one-rank SUM is the identity: the nets must equal the plain run's)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs-total", type=int, default=2048)
ap.add_argument("--out", required=True)
ap.add_argument("--nccl-world1", action="store_true")
a = ap.parse_args()
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
torch.cuda.set_device(0)
if a.nccl_world1:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29900 + os.getpid() % 90))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from mhppo import ppo  # noqa: E402
    ppo.set_force_collectives(True)  # the update's collectives run (one rank: identity sums)
elif world > 1:
    dist.init_process_group("gloo")  # rehearsal: the ranks share the box's one GPU
from mhppo.algo import Algo_PPO  # noqa: E402
from mhppo.env import VecCrosswalk  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

n = a.envs_total // world
venv = VecCrosswalk("4cars", n, 4, 1, 2, seed_base=11, env_id_offset=rank * n, device="cuda:0")
torch.manual_seed(0)
algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=3)
algo.train(1)
if rank == 0:
    np.save(a.out, np.concatenate([net.flat().cpu().numpy() for net in algo.nets()]))
if dist.is_initialized():
    dist.barrier()
    dist.destroy_process_group()
