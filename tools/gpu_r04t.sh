#!/bin/bash
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O/prof2
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_bucket_scatter_gpu.py tests/test_train_gpu.py tests/test_checkpoint_gpu.py tests/test_bugfix_gpu.py tests/test_dp_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for cfg in 2 2; do
  timeout -k 10 240 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/b$cfg.json 2> $O/b$cfg.err || { tail -20 $O/b$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b$cfg.json').read().strip().splitlines()[-1]);print('cfg $cfg', round(d['ms_per_step'],3), round(d['value']/1e6,2))" | tee -a $O/summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof2 -o run -- python3 bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
