#!/bin/bash
# Config 2 (BASELINE.json configs[1]: coop 2/1/2, 4096 envs) bench line + rocprofv3 kernel stats +
# PMC HBM traffic, one GPU call: bash tools/gpu_cfg2.sh <tag>
set -o pipefail
TAG=${1:-cfg2}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_pmc.sh $TAG/pmc 2 --envs 4096 || exit 1
cp $OUT/pmc/traffic.json profiles/pmc_traffic_cfg2.json
timeout -k 10 400 python -u bench.py --config 2 --envs 4096 --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config 2 --envs 4096 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo PROF FAILED; tail -30 $OUT/prof.err; exit 1; }
cp profiles/pmc_traffic_cfg2.json $OUT/
