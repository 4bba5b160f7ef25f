#!/bin/bash
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O/prof3
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof3 -o run -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof3.log 2>&1 || { tail -20 $O/prof3.log; exit 1; }
tail -1 $O/prof3.log
