#!/bin/bash
# One GPU box session: parity suite, smoke, bench, rocprofv3 kernel stats.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag> [tests|bench|all] [pytest args...]
set -o pipefail
TAG=${1:-run}; WHAT=${2:-all}; shift 2; ARGS=${@:-tests}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
  timeout -k 10 900 python -u -m pytest $ARGS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
  timeout -k 10 400 python -u bench.py --config 4 --no-cpu-baseline > $OUT/bench_cfg4.json 2> $OUT/bench_cfg4.err || { echo BENCH4 FAILED; tail -30 $OUT/bench_cfg4.err; exit 1; }
  cat $OUT/bench_cfg4.json
fi
if [ "$WHAT" = prof ] || [ "$WHAT" = all ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo PROF FAILED; tail -30 $OUT/prof.err; exit 1; }
  find $OUT/prof -name '*kernel_stats.csv' | head -3
fi
