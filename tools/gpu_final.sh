#!/bin/bash
# End-of-session GPU record: parity suite + smoke + bench (cfg3, cfg4) + rocprofv3 kernel stats,
# then the HBM-traffic PMC passes of cfg3 and cfg4 (tools/gpu_pmc.sh).  usage: bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
bash tools/gpu_check.sh $TAG all || exit 1
bash tools/gpu_pmc.sh $TAG/pmc3 3 || exit 1
bash tools/gpu_pmc.sh $TAG/pmc4 4 || exit 1
