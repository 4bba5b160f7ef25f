#!/bin/bash
# Interleaved A/B of environment-variable settings on the driver's bench command:
# usage (via gpurun): bash tools/ab_env_vars.sh <tag> <reps> <config> "<VAR=val ...>" ...  ("-" = none)
set -o pipefail
TAG=$1; REPS=$2; CFG=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq $REPS); do
  i=0
  for v in "$@"; do
    i=$((i+1)); f=$O/abv_${i}_cfg${CFG}_$r.json
    if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline > $f 2> $O/abv_${i}_$r.err || { tail -20 $O/abv_${i}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];s=d['rollout_step_us'];it=d['iter_ms'];print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,2), 'M/s train', round(r['launch_ms'],4), 'ms step product', round(s['product'],1), 'parts', round(s.get('parts',0),1), 'one_chain', round(s['one_chain'],1), 'us iters', min(it), '..', max(it))" $f "[$v]#$r" | tee -a $O/abv_summary.txt
  done
done
exit 0
