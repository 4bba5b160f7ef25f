#!/bin/bash
# r04: two-part rollout parity + A/B (parts 1 vs 2) of the headline bench; x3 prefetch depth A/B
set -o pipefail
OUT=gpurun_out/r04i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_rollout_gpu.py tests/test_rollout_fullscale_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for pp in 2 1; do
  MHPPO_ROLLOUT_PARTS=$pp timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_cfg3_parts$pp.json 2> $OUT/bench_cfg3_parts$pp.err || { tail -20 $OUT/bench_cfg3_parts$pp.err; exit 1; }
done
MHPPO_ROLLOUT_PARTS=2 timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_cfg4_parts2.json 2> $OUT/bench_cfg4.err || exit 1
bash tools/ab_x3.sh base pf2 base pf2 > $OUT/ab_pf2.txt 2>&1 || exit 1
exit 0
