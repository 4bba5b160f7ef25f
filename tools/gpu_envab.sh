#!/bin/bash
# Env-kernel change check in one GPU call: GPU suite on the in-tree library, env phases of the
# timing build, rollout A/B against build_ab/base.  Usage: bash tools/gpu_envab.sh <tag> [pytest paths]
set -o pipefail
TAG=${1:-envab}; shift; ARGS=${@:-tests}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
MHPPO_LIB=build_ab/timing/libmhppo.so timeout -k 10 120 python tools/env_phases.py 4cars 4 1 2 65536 > $OUT/env_phases.txt 2>&1 || { tail -20 $OUT/env_phases.txt; exit 1; }
cat $OUT/env_phases.txt
bash tools/ab_env.sh ${ABV:-base new} > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
