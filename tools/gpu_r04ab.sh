#!/bin/bash
set -o pipefail
O=gpurun_out/r04ac; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ppo_gpu.py tests/test_update_scale_gpu.py tests/test_train_gpu.py tests/test_bugfix_gpu.py tests/test_checkpoint_gpu.py tests/test_dp_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB_ARGS="--pair" bash tools/ab_x3.sh base a62 c14 base a62 c14 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
grep -v amdgpu.ids $O/ab.txt
for cfg in 3 4 2; do
timeout -k 10 240 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/b$cfg.json 2> $O/b$cfg.err || { tail -20 $O/b$cfg.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b$cfg.json').read().strip().splitlines()[-1]);print('cfg$cfg', round(d['ms_per_step'],3), round(d['value']/1e6,2), round(d['roofline']['launch_ms'],4), round(d['roofline']['frac'],4))"
done
