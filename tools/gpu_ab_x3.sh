#!/bin/bash
# Train-kernel A/B: the in-tree library (base) against build_ab/<variant>, with the parity tests
# that pin the kernel run on the variant.  usage: bash tools/gpu_ab_x3.sh <variant>
set -o pipefail
V=${1:?variant}; OUT=gpurun_out/abx3; mkdir -p $OUT
MHPPO_LIB=build_ab/$V/libmhppo.so timeout -k 10 600 python -u -m pytest tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_update_scale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_x3.sh base $V base $V base $V
