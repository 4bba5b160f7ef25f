#!/bin/bash
# r04: per-block partial fold + fused policy/env step — parity tests, micro-bench, fused vs unfused
# bench lines on configs 3/4/2, config-4 PMC passes, config-2 rocprof
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_rollout_gpu.py tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_update_scale_gpu.py tests/test_bugfix_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 120 python -u tools/bench_mlp_train.py --reps 10 --pair --choice 27 --choice-rows 262144 > $O/mlp.txt 2>&1 || { cat $O/mlp.txt; exit 1; }
cat $O/mlp.txt
timeout -k 10 120 python -u tools/bench_mlp_train.py --rows 327680 --reps 20 --pair > $O/mlp_small.txt 2>&1 || { cat $O/mlp_small.txt; exit 1; }
cat $O/mlp_small.txt
for cfg in 3 4 2; do
  for fz in 1 0; do
    MHPPO_ROLLOUT_FUSED=$fz timeout -k 10 240 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $O/b${cfg}_f$fz.json 2> $O/b${cfg}_f$fz.err || { tail -20 $O/b${cfg}_f$fz.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/b${cfg}_f$fz.json').read().strip().splitlines()[-1]);print('cfg $cfg fused $fz', round(d['ms_per_step'],2), round(d['value']/1e6,2), d['rollout_step_us'], round(d['roofline']['launch_ms'],4))" | tee -a $O/summary.txt
  done
done
bash tools/gpu_pmc.sh r04m/pmc4 4
mkdir -p $O/prof2 && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof2 -o run -- python3 bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
tail -1 $O/prof2.log
