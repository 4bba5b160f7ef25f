#!/bin/bash
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O/prof2
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof2 -o run -- python3 bench.py --config 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof2.log 2>&1 || { tail -20 $O/prof2.log; exit 1; }
tail -1 $O/prof2.log
