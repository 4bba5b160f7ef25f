#!/bin/bash
# Train-kernel A/B against build_ab/prev with the parity tests that pin it.
set -o pipefail
OUT=gpurun_out/abx3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_update_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_x3.sh base prev rt base prev rt
