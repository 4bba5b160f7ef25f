#!/bin/bash
# r04: config 2 (coop 2/1/2, 4 096 envs): bench lines (fused step off / on), rocprof kernel trace
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
export PYTHONUNBUFFERED=1
for fz in 0 1 0 1; do
  MHPPO_ROLLOUT_FUSED=$fz timeout -k 10 240 python -u bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $O/b2_f$fz.json 2> $O/b2_f$fz.err || { tail -20 $O/b2_f$fz.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b2_f$fz.json').read().strip().splitlines()[-1]);print('cfg 2 fused $fz', round(d['ms_per_step'],3), round(d['value']/1e6,2), {k: (round(v,1) if isinstance(v,float) else v) for k,v in d['rollout_step_us'].items() if k!='note'}, round(d['roofline']['launch_ms'],4))" | tee -a $O/summary.txt
done
mkdir -p $O/prof2 && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
tail -1 $O/prof2.log
