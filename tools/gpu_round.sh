#!/bin/bash
# Round check + env-kernel diagnostics in one GPU call: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
bash tools/gpu_check.sh $TAG all || exit 1
MHPPO_LIB=build_ab/timing/libmhppo.so timeout -k 10 120 python tools/env_phases.py 4cars 4 1 2 65536 > gpurun_out/$TAG/env_phases.txt 2>&1 || { tail -20 gpurun_out/$TAG/env_phases.txt; exit 1; }
cat gpurun_out/$TAG/env_phases.txt
bash tools/env_pmc.sh $TAG/envpmc
