#!/bin/bash
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_bucket_scatter_gpu.py tests/test_train_gpu.py tests/test_checkpoint_gpu.py tests/test_bugfix_gpu.py tests/test_dp_gpu.py tests/test_rollout_fullscale_gpu.py tests/test_nan_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for cfg in 2 2 3 4; do
  timeout -k 10 240 python -u bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline > $O/b$cfg.json 2> $O/b$cfg.err || { tail -20 $O/b$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b$cfg.json').read().strip().splitlines()[-1]);print('cfg $cfg', round(d['ms_per_step'],3), round(d['value']/1e6,2))" | tee -a $O/summary.txt
done
