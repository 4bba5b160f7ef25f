#!/bin/bash
set -o pipefail
O=gpurun_out/r04ae; mkdir -p $O
export PYTHONUNBUFFERED=1
for cfg in 3 4 2; do
timeout -k 10 240 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/b${cfg}.json 2> $O/b${cfg}.err || { tail -20 $O/b${cfg}.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b${cfg}.json').read().strip().splitlines()[-1]);r=d['roofline'];print('cfg$cfg', round(d['ms_per_step'],3), round(d['value']/1e6,2), round(r['launch_ms'],4), round(r['frac'],4), r['launches'], r['measured_on'])"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dp_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
