#!/bin/bash
set -o pipefail
O=gpurun_out/r04af; mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in 3 4; do for k in 2 3 4 2 3 4; do
MHPPO_ROLLOUT_PARTS=$k timeout -k 10 240 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/b${cfg}_$k.json 2> $O/b${cfg}_$k.err || { tail -20 $O/b${cfg}_$k.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b${cfg}_$k.json').read().strip().splitlines()[-1]);r=d['rollout_step_us'];print('cfg$cfg parts $k', round(d['ms_per_step'],3), round(d['value']/1e6,2), round(r['parts'],1), round(r['product'],1))"
done; done
