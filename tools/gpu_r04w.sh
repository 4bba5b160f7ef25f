#!/bin/bash
set -o pipefail
bash tools/gpu_pmc.sh r04w/pmc3 3 && bash tools/gpu_pmc.sh r04w/pmc4 4 && bash tools/gpu_pmc.sh r04w/pmc2 2
