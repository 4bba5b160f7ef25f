#!/bin/bash
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_rollout_gpu.py tests/test_train_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for g in 1 0 1 0; do
  MHPPO_ROLLOUT_GRAPH=$g timeout -k 10 240 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > $O/b3_g$g.json 2> $O/b3_g$g.err || { tail -20 $O/b3_g$g.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b3_g$g.json').read().strip().splitlines()[-1]);print('cfg3 graph $g', round(d['ms_per_step'],3), round(d['value']/1e6,2), {k: (round(v,1) if isinstance(v,float) else v) for k,v in d['rollout_step_us'].items() if k!='note'})" | tee -a $O/summary.txt
done
