#!/bin/bash
# r04: choice heads on the bf16x3 split kernel — parity tests, micro-bench, cfg3 bench
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_update_scale_gpu.py tests/test_bugfix_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 120 python -u tools/bench_mlp_train.py --reps 10 --choice 27 --choice-rows 262144 > $O/mlp.txt 2>&1 || { cat $O/mlp.txt; exit 1; }
cat $O/mlp.txt
timeout -k 10 120 python -u tools/bench_mlp_train.py --rows 100000 --reps 20 --choice 17 --choice-rows 1048576 > $O/mlp17.txt 2>&1 || { cat $O/mlp17.txt; exit 1; }
cat $O/mlp17.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
