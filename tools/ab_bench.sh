#!/bin/bash
# Interleaved A/B of library builds on the driver's bench command (bench.py --steps 20 --warmup 5):
# usage (via gpurun, from the repo root): bash tools/ab_bench.sh <tag> <reps> <config> <variant>...
# variant: base (the in-tree library) or a build_ab/<v>/libmhppo.so (tools/ab_build.sh <v> "<flags>").
# One summary line per run (ms per iteration, train launch, env kernel, the iteration-time spread).
set -o pipefail
TAG=$1; REPS=$2; CFG=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq $REPS); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="build_ab/$v/libmhppo.so"; fi
    f=$O/ab_${v}_cfg${CFG}_$r.json
    MHPPO_LIB=$lib timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline > $f 2> $O/ab_${v}_$r.err || { tail -20 $O/ab_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];e=d['roofline_env'];it=d['iter_ms'];print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,2), 'M/s train', round(r['launch_ms'],4), 'ms env', round(e['kernel_ms']*1e3,2), 'us iters', min(it), '..', max(it))" $f "$v#$r" | tee -a $O/ab_summary.txt
  done
done
exit 0
