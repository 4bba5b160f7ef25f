#!/bin/bash
# HBM traffic per kernel launch: separate FETCH_SIZE and WRITE_SIZE rocprofv3 passes over a
# short bench run, summarised by tools/pmc_summary.py (gfx950 read correction applied there).
# Usage (via gpurun, from the repo root): bash tools/gpu_pmc.sh <tag> [config] [extra bench args]
# -> gpurun_out/<tag>/traffic.json; bench.py reads it as profiles/pmc_traffic_cfg<config>.json
set -o pipefail
OUT=gpurun_out/${1:-pmc}; CFG=${2:-3}; shift 2; EXTRA="$@"; mkdir -p $OUT
export TMPDIR=/tmp
# one-chain rollout: every env-step launch covers all N envs (the bench's env roofline is per full launch)
export MHPPO_ROLLOUT_PARTS=1
for c in FETCH_SIZE WRITE_SIZE; do
  d=$OUT/$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $d -o run -- python3 bench.py --config $CFG $EXTRA --no-cpu-baseline --steps 1 --warmup 1 > $d.log 2>&1 || { echo "PMC $c FAILED"; tail -20 $d.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/fetch $OUT/write $OUT/traffic.json && echo PMC OK
