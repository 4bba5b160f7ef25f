#!/bin/bash
# Interleaved A/B of library builds on tools/bench_rollout.py (80-step collects, the product's parts):
# usage (via gpurun): bash tools/ab_rollout.sh <tag> <reps> "<ROLLOUT_CFG>" <variant>...
set -o pipefail
TAG=$1; REPS=$2; CFG=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq $REPS); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
    MHPPO_LIB=$lib ROLLOUT_CFG="$CFG" timeout -k 10 200 python -u tools/bench_rollout.py > $O/${v}_$r.txt 2>&1 || { tail -20 $O/${v}_$r.txt; exit 1; }
    echo "$v#$r $(grep 'iter 2' $O/${v}_$r.txt)" | tee -a $O/summary.txt
  done
done
exit 0
