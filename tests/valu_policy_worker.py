"""One rollout episode per case on the VALU reference policy kernels, saved for
tests/test_rollout_gpu.py::test_mfma_policy_bit_identical_to_valu.  Runs in its own process
with MHPPO_LIB=tests/lib/libmhppo_test.so (the test build: the shipped library has the MFMA
policy kernel only).

usage: MHPPO_LIB=tests/lib/libmhppo_test.so python tests/valu_policy_worker.py <out.npz> <mode> <case>...
mode: sorted (k_policy_sorted) or unsorted (k_policy); case: variant,nb_car,nb_ped,nb_lines"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd"), os.path.dirname(os.path.abspath(__file__))]
import numpy as np  # noqa: E402

from rollout_policy_case import run_case  # noqa: E402

out, mode, cases = sys.argv[1], sys.argv[2], sys.argv[3:]
res = {}
for cs in cases:
    v, nc, npd, nl = cs.split(",")
    for k, x in run_case((v, int(nc), int(npd), int(nl)), True if mode == "sorted" else "unsorted").items():
        res[f"{cs}/{k}"] = x
np.savez(out, **res)
