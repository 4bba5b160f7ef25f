#!/bin/bash
# A/B of the env-step kernel across build_ab variants: rollout collect time (tools/bench_rollout.py)
set -o pipefail
for round in 1 2; do
  for v in "$@"; do
    if [ "$v" = new ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
    echo "== $v (round $round)"
    MHPPO_LIB=$lib timeout -k 10 120 python tools/bench_rollout.py || exit 1
  done
done
