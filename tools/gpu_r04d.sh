#!/bin/bash
# r04 A/B: headline bench (cfg3) and config 2 with the fused actor/critic pair launch on and off,
# plus a host-side cProfile of the config-2 iteration.  usage: bash tools/gpu_r04d.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-r04d}; mkdir -p $OUT
for pp in 1 0; do
  MHPPO_PIPELINE_PAIRS=$pp timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_cfg3_pp$pp.json 2> $OUT/bench_cfg3_pp$pp.err || exit 1
  MHPPO_PIPELINE_PAIRS=$pp timeout -k 10 300 python -u bench.py --config 2 --envs 4096 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_cfg2_pp$pp.json 2> $OUT/bench_cfg2_pp$pp.err || exit 1
done
timeout -k 10 300 python -u -m cProfile -s tottime bench.py --config 2 --envs 4096 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/cprofile_cfg2.txt 2>&1 || exit 1
exit 0
