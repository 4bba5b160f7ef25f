#!/bin/bash
set -o pipefail
O=gpurun_out/r04ag; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ppo_gpu.py tests/test_update_scale_gpu.py tests/test_train_gpu.py tests/test_bugfix_gpu.py tests/test_checkpoint_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB_EXACT=1 AB_ARGS="--pair" bash tools/ab_x3.sh base dmapred base dmapred > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
