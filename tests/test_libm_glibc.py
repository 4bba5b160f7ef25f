"""The policy heads' float transcendentals restated (mh-ppo_amd/csrc/libm_glibc.h) against this
host's glibc, over EVERY float input: tanhf (the continuous heads, Model_PPO :87-89, through
ATen's scalar tail loop for the reference's batch-1 rollout forward), its expm1f, and expf (the
choice head's softmax as the oracle restates it, oracle/rollout_oracle.c).  The device compiles
the same source (tests/test_libm_gpu.py pins the device side), so GPU == glibc bit for bit."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_libm_restatement_matches_glibc_on_all_floats():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tools")])
    env = dict(os.environ, OMP_NUM_THREADS=str(min(8, os.cpu_count() or 1)))
    r = subprocess.run([os.path.join(ROOT, "tools", "libm_check")], capture_output=True, text=True, env=env,
                       timeout=600)
    res = json.loads(r.stdout)
    assert res["checked"] == 1 << 32
    for fn in ("tanhf", "expm1f", "expf"):
        assert res[fn]["mismatches"] == 0, res
    assert r.returncode == 0
