#!/bin/bash
# A/B of the split-precision train kernel across environment switches of the in-tree library:
# usage: bash tools/ab_x3env.sh "VAR=.. VAR=.." "VAR=.." ...   (each argument one variant)
set -o pipefail
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/bench_mlp_train.py --reps 10 || exit 1
done
