"""(usage: dp_diff.py [rep])  Max |nets(2 ranks x 1024 envs) - nets(1 rank x 2048 envs)| after one bench iteration (the check of
tests/test_dp_gpu.py::test_bench_launches_two_ranks, printed instead of asserted)."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = tempfile.mkdtemp()
one, two = os.path.join(d, "one.npy"), os.path.join(d, "two.npy")
env = dict(os.environ, OMP_NUM_THREADS="4")
env.pop("WORLD_SIZE", None)
common = ["--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--dist-backend", "gloo"]
subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--envs", "2048", "--save-nets", one]
               + common, check=True, timeout=300, env=env, cwd=d, capture_output=True)
if sys.argv[1:] == ["rep"]:  # run-to-run: the one-rank run again
    subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--envs", "2048", "--save-nets",
                    two] + common, check=True, timeout=300, env=env, cwd=d, capture_output=True)
else:
    subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--envs", "1024", "--save-nets",
                    two] + common, check=True, timeout=300, env=env, cwd=d, capture_output=True)
a, b = np.load(one), np.load(two)
e = np.abs(a - b)
print(f"n {a.size}  max {e.max():.3g}  >1e-5: {(e > 1e-5).sum()}  >1e-6: {(e > 1e-6).sum()}  median {np.median(e):.3g}")
