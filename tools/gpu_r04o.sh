#!/bin/bash
# r04: split train kernel per-launch fixed cost (tiles-per-wave sweep) + rocprof of the sweep
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_mlp_train.py --sweep --reps 20 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
cat $O/sweep.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_mlp_train.py --sweep --reps 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
