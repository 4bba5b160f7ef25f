#!/bin/bash
# rocprofv3 kernel stats of short benches across library builds (kernel-time A/B of small kernels):
# usage (via gpurun): bash tools/prof_variants.sh <tag> <config> <kernel-substring> <variant>...
# (base = the in-tree library, else build_ab/<v>/libmhppo.so)
set -o pipefail
TAG=$1; CFG=$2; PAT=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
  MHPPO_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_${v}_$CFG -o run -- python3 bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 1 > $O/p_${v}_$CFG.log 2>&1 || { tail -20 $O/p_${v}_$CFG.log; exit 1; }
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r['Name']: print(sys.argv[3], r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')" $O/p_${v}_$CFG/run_kernel_stats.csv "$PAT" "$v" | tee -a $O/prof_variants.txt
done
exit 0
