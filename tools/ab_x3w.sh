#!/bin/bash
# split-precision train kernel: 4 vs 8 waves per block (MHPPO_X3_WAVES) on the in-tree library
set -o pipefail
for w in 4 8; do
  echo "== waves=$w"
  MHPPO_X3_WAVES=$w timeout -k 10 120 python tools/bench_mlp_train.py --reps 10 || exit 1
done
