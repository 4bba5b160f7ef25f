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


def test_bench_launches_two_ranks(tmp_path):
    """`bench.py --gpus 2` starts its own two ranks (torch.distributed.run, gloo rehearsal on
    the box's one GPU), reports n_gpus 2 and the world's env ranges, and its two ranks of
    1024 envs train the same nets as one rank of 2048 envs (global-id env streams and noise)."""
    import json
    one, two = str(tmp_path / "one.npy"), str(tmp_path / "two.npy")
    env = dict(os.environ, OMP_NUM_THREADS="4")
    env.pop("WORLD_SIZE", None)
    common = ["--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--dist-backend", "gloo"]
    out1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--envs", "2048",
                           "--save-nets", one] + common, check=True, timeout=300, env=env, cwd=tmp_path,
                          capture_output=True, text=True).stdout
    out2 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--envs", "1024",
                           "--save-nets", two] + common, check=True, timeout=300, env=env, cwd=tmp_path,
                          capture_output=True, text=True).stdout
    l1 = json.loads([x for x in out1.splitlines() if x.startswith("{")][-1])
    l2 = json.loads([x for x in out2.splitlines() if x.startswith("{")][-1])
    assert l1["n_gpus"] == 1 and l2["n_gpus"] == 2
    assert l2["dist"]["world_size"] == 2 and l2["dist"]["env_ranges"] == [[0, 1024], [1024, 2048]]
    a, b = np.load(one), np.load(two)
    assert np.isfinite(a).all()
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-5)


def test_rccl_collectives_one_rank(tmp_path):
    """The update's RCCL path (backend "nccl", device-bound init, the advantage-sum / gradient-
    bucket / count all-reduces on device tensors) exercised on the one-GPU box: one rank with the
    collectives forced on trains the same nets as the plain process (a one-rank SUM is the
    identity; 1e-6 absolute leaves room only for a summation-order difference)."""
    one, rc = str(tmp_path / "one.npy"), str(tmp_path / "rccl.npy")
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    subprocess.run([sys.executable, WORKER, "--envs-total", "1024", "--out", one], check=True, timeout=240,
                   env=env, cwd=tmp_path)
    subprocess.run([sys.executable, WORKER, "--envs-total", "1024", "--out", rc, "--nccl-world1"], check=True,
                   timeout=240, env=env, cwd=tmp_path)
    a, b = np.load(one), np.load(rc)
    assert np.isfinite(a).all()
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-6)


def test_bench_force_collectives_rccl(tmp_path):
    """`bench.py --force-collectives` on one GPU: a one-rank RCCL group with every data-parallel
    collective of the product's update issued (ppo.set_force_collectives, no monkey-patching)
    trains the same nets as the plain run."""
    import json
    one, rc = str(tmp_path / "one.npy"), str(tmp_path / "rc.npy")
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    common = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--envs", "1024", "--steps", "1",
              "--warmup", "0", "--no-cpu-baseline"]
    subprocess.run(common + ["--save-nets", one], check=True, timeout=300, env=env, cwd=tmp_path,
                   capture_output=True, text=True)
    out = subprocess.run(common + ["--save-nets", rc, "--force-collectives"], check=True, timeout=300, env=env,
                         cwd=tmp_path, capture_output=True, text=True).stdout
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    assert line["dist"]["backend"] == "nccl" and line["dist"]["collectives"].startswith("forced")
    a, b = np.load(one), np.load(rc)
    assert np.isfinite(a).all()
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-6)
