#!/bin/bash
set -o pipefail
O=gpurun_out/r04ah; mkdir -p $O
export PYTHONUNBUFFERED=1
for i in 1 2; do for cfg in 3 2; do
timeout -k 10 240 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/b${cfg}_$i.json 2> $O/b${cfg}_$i.err || { tail -20 $O/b${cfg}_$i.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b${cfg}_$i.json').read().strip().splitlines()[-1]);print('cfg$cfg', round(d['ms_per_step'],3), round(d['value']/1e6,2), round(d['roofline']['launch_ms'],4), round(d['roofline']['frac'],4))"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
