#!/bin/bash
# A/B of the env-step kernel across library builds (tools/env_steps.py mean per-step duration,
# configs 3 and 4): usage: bash tools/ab_env.sh <variant>... (base = the in-tree library, else
# build_ab/<v>/libmhppo.so, built by tools/ab_build.sh <v> "<flags>")
set -o pipefail
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
  for cfg in "4cars 4 1 2" "scalable 8 1 4"; do
    echo "== $v $cfg"
    MHPPO_LIB=$lib ROLLOUT_CFG="$cfg" timeout -k 10 120 python tools/env_steps.py > gpurun_out/ab_env_step.txt 2>&1 || exit 1
    grep "mean" gpurun_out/ab_env_step.txt
  done
done
exit 0
