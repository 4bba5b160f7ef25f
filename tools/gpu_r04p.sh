#!/bin/bash
# r04: early first-tile DMA, one-launch block reduction, train_epochs launch plans — tests + benches
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_rollout_gpu.py tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_update_scale_gpu.py tests/test_bugfix_gpu.py tests/test_dp_gpu.py tests/test_checkpoint_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 python -u tools/bench_mlp_train.py --sweep --reps 20 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
cat $O/sweep.txt
for cfg in 2 3 4; do
  timeout -k 10 240 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline > $O/b$cfg.json 2> $O/b$cfg.err || { tail -20 $O/b$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b$cfg.json').read().strip().splitlines()[-1]);print('cfg $cfg', round(d['ms_per_step'],3), round(d['value']/1e6,2), round(d['roofline']['launch_ms'],4), round(d['roofline']['frac'],4), round(d['roofline_env']['frac'],4), {k: (round(v,1) if isinstance(v,float) else v) for k,v in d['rollout_step_us'].items() if k!='note'})" | tee -a $O/summary.txt
done
