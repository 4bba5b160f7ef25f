#!/bin/bash
# r04 round record: full GPU suite, smoke, default bench (cfg3, with cpu_baseline), cfg4 and cfg2 lines,
# rocprof kernel stats of the default bench, PMC traffic passes for cfg3
set -o pipefail
O=gpurun_out/${R04_TAG:-r04_final}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { tail -20 $O/bench_cfg4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > $O/bench_cfg2.json 2> $O/bench_cfg2.err || { tail -20 $O/bench_cfg2.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
bash tools/gpu_pmc.sh ${R04_TAG:-r04_final}/pmc3 3
