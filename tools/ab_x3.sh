#!/bin/bash
# A/B of the split-precision train kernel: build variants x waves, plus the exact f32 kernel
set -o pipefail
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
  for w in 8 4; do
    echo "== $v waves=$w"
    MHPPO_X3_WAVES=$w MHPPO_LIB=$lib timeout -k 10 120 python tools/bench_mlp_train.py --reps 10 || exit 1
  done
done
echo "== exact f32"
timeout -k 10 120 python tools/bench_mlp_train.py --reps 10 --exact || exit 1
