#!/bin/bash
# policy-kernel A/B: the rollout parity tests on build_ab/<variant>, then tools/bench_rollout.py
# (per-kernel HIP-event times) alternated base / variant.  usage: bash tools/gpu_ab_policy.sh <variant>
set -o pipefail
V=${1:?variant}; OUT=gpurun_out/abpol; mkdir -p $OUT
MHPPO_LIB=build_ab/$V/libmhppo.so timeout -k 10 600 python -u -m pytest tests/test_rollout_gpu.py tests/test_rollout_fullscale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in base $V; do
    if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
    echo "== $v"
    MHPPO_LIB=$lib timeout -k 10 200 python3 tools/bench_rollout.py > $OUT/roll_$v.txt 2>&1 || { tail -5 $OUT/roll_$v.txt; exit 1; }
    cat $OUT/roll_$v.txt | grep -v amdgpu.ids
  done
done
