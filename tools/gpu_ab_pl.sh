#!/bin/bash
# A/B of the permlane32_swap change (train + policy kernels) against build_ab/prev, with the
# parity tests that pin both kernels.
set -o pipefail
OUT=gpurun_out/pl; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rollout_gpu.py tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_update_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for v in base prev base prev; do
  if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
  echo "== $v rollout"
  MHPPO_LIB=$lib timeout -k 10 200 python3 tools/bench_rollout.py > $OUT/roll_$v.txt 2>&1 || { tail -5 $OUT/roll_$v.txt; exit 1; }
  grep "iter" $OUT/roll_$v.txt
done
