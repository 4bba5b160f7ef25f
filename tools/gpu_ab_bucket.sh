#!/bin/bash
# bucket-scatter A/B: parity test on each variant, then base / variants alternated x3.
# usage: bash tools/gpu_ab_bucket.sh <variant>...
set -o pipefail
OUT=gpurun_out/abbk; mkdir -p $OUT
for V in "$@"; do
  MHPPO_LIB=build_ab/$V/libmhppo.so timeout -k 10 300 python -u -m pytest tests/test_bucket_scatter_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$V.log 2>&1 || { tail -30 $OUT/pytest_$V.log; exit 1; }
  echo "$V: $(tail -1 $OUT/pytest_$V.log)"
done
for r in 1 2 3; do
  TAG=base timeout -k 10 120 python tools/bench_bucket.py || exit 1
  for V in "$@"; do TAG=$V MHPPO_LIB=build_ab/$V/libmhppo.so timeout -k 10 120 python tools/bench_bucket.py || exit 1; done
done
