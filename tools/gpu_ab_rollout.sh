set -o pipefail
OUT=gpurun_out/r02_v; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rollout_gpu.py tests/test_eval_gpu.py tests/test_nan_gpu.py tests/test_train_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_env.sh prev new > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
grep -E "==|iter 2" $OUT/ab.txt
