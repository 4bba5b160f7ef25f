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
    python3 -c "import re,sys;v=[float(m.group(2)) for m in re.finditer(r'step +(\\d+): +([\\d.]+) us', open(sys.argv[1]).read()) if 2<=int(m.group(1))<=18];print('  steps 2-18 mean %.1f us, max %.1f' % (sum(v)/len(v), max(v)))" gpurun_out/ab_env_step.txt
  done
done
exit 0
