#!/bin/bash
set -o pipefail
O=gpurun_out/r04ad; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ppo_gpu.py tests/test_update_scale_gpu.py tests/test_train_gpu.py tests/test_bugfix_gpu.py tests/test_checkpoint_gpu.py tests/test_dp_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for cfg in 3 2; do for ts in 2 1 2 1; do
MHPPO_TRAIN_STREAMS=$ts timeout -k 10 240 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/b${cfg}_$ts.json 2> $O/b${cfg}_$ts.err || { tail -20 $O/b${cfg}_$ts.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b${cfg}_$ts.json').read().strip().splitlines()[-1]);print('cfg$cfg streams $ts', round(d['ms_per_step'],3), round(d['value']/1e6,2), round(d['roofline']['launch_ms'],4))"
done; done
