#!/bin/bash
# Round-3 session-3 GPU call: parity suite + smoke + bench (cfg3, cfg4) + rocprof kernel stats,
# then the train-kernel A/B of compiler post-RA scheduling variants (tools/ab_x3.sh).
# usage: bash tools/gpu_r03s3.sh <tag> [ab variants...]
set -o pipefail
TAG=${1:-r03s3}; shift
bash tools/gpu_check.sh $TAG all || exit 1
[ $# -gt 0 ] && { bash tools/ab_x3.sh "$@" > gpurun_out/$TAG/ab_x3.txt 2>&1 || { tail -20 gpurun_out/$TAG/ab_x3.txt; exit 1; }; cat gpurun_out/$TAG/ab_x3.txt; }
exit 0
