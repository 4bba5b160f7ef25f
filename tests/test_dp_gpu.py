"""Data parallel on the real HIP path: 2 ranks (torchrun, gloo, sharing the box's one GPU)
each training on half of 2048 envs give the same nets as one process on all 2048 envs.
The rollout is shard-invariant (global-id streams); the update all-reduces the advantage
sums and the flat gradients, so the weights agree up to float32 summation order."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_worker.py")


def test_two_ranks_equal_one_process(tmp_path):
    one, two = str(tmp_path / "one.npy"), str(tmp_path / "two.npy")
    env = dict(os.environ, OMP_NUM_THREADS="4")
    # cwd: Algo_PPO.train writes its reward curves to ./load_model/parameters, as the reference
    subprocess.run([sys.executable, WORKER, "--out", one], check=True, timeout=240, env=env, cwd=tmp_path)
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(29600 + os.getpid() % 300), WORKER,
                    "--out", two], check=True, timeout=240, env=env, cwd=tmp_path)
    a, b = np.load(one), np.load(two)
    assert a.shape == b.shape
    assert np.isfinite(a).all()
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-5)
