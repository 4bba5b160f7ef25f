#!/bin/bash
# A/B of the split-precision train kernel across library builds, plus the exact f32 kernel:
# usage: bash tools/ab_x3.sh <variant>... (base = the in-tree library, else build_ab/<v>/libmhppo.so,
# built by tools/ab_build.sh <v> "<flags>")
set -o pipefail
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
  echo "== $v split"
  MHPPO_LIB=$lib timeout -k 10 120 python tools/bench_mlp_train.py --reps 10 $AB_ARGS || exit 1
  if [ -n "$AB_EXACT" ]; then
    echo "== $v exact f32"
    MHPPO_LIB=$lib timeout -k 10 120 python tools/bench_mlp_train.py --reps 10 --exact || exit 1
  fi
done
exit 0
