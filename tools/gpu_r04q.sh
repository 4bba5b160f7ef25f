#!/bin/bash
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/host_profile.py 2 10 > $O/host2.txt 2>&1 || { tail -30 $O/host2.txt; exit 1; }
head -3 $O/host2.txt
timeout -k 10 300 python -u tools/host_profile.py 3 3 > $O/host3.txt 2>&1 || { tail -30 $O/host3.txt; exit 1; }
head -3 $O/host3.txt
