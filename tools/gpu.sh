#!/bin/bash
# One parametrised GPU session (replaces the per-experiment gpu_r0*.sh one-offs).
# usage (from the repo root, via gpurun):
#   bash tools/gpu.sh <tag> <step>[,<step>...] ...
# steps (each under its own time limit; the first failure ends the session):
#   tests[=file:file...]   pytest -m gpu (all GPU tests, or the listed files under tests/)
#   smoke                  __graft_entry__.smoke()
#   bench=<cfg>[:<n>]      bench.py --config <cfg> (n repeats, one summary line each; cfg 3 with cpu_baseline
#                          only when named "bench=3full")
#   ab=<v>:<v>...          tools/ab_x3.sh over the A/B library variants (AB_ARGS passed through)
#   mlp                    tools/bench_mlp_train.py (AB_ARGS passed through) on the in-tree library
#   prof=<cfg>             rocprofv3 --kernel-trace --stats of bench.py --config <cfg>
#   pmc=<cfg>              FETCH_SIZE / WRITE_SIZE passes of bench.py --config <cfg> (tools/gpu_pmc.sh)
#   envsteps=<v_c_p_l>     per-step env kernel durations (tools/env_steps.py), e.g. envsteps=4cars_4_1_2
#   py=<script>[:args]     python tools/<script> with args (':' separated), output to <tag>/<script>.txt
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
summ() {  # one summary line of a bench JSON
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];e=d['roofline_env'];print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,2), 'M/s train', round(r['launch_ms'],4), 'ms', round(r['frac'],4), 'env', round(e['kernel_ms']*1e3,2), 'us', round(e['frac'],4), 'step', round(d['rollout_step_us']['product'],1), 'us', 'iters', min(d.get('iter_ms',[0])), '..', max(d.get('iter_ms',[0])))" "$1" "$2"
}
for arg in "$@"; do for step in ${arg//,/ }; do
  key=${step%%=*}; val=${step#*=}; [ "$key" = "$step" ] && val=""
  case $key in
    tests)
      files=tests; [ -n "$val" ] && files=$(echo $val | tr ':' '\n' | sed 's|^|tests/|' | tr '\n' ' ')
      timeout -k 10 1100 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 $O/pytest_gpu.log; exit 1; }
      tail -1 $O/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail -30 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      cfg=${val%%:*}; n=${val#*:}; [ "$n" = "$val" ] && n=1
      extra="--no-cpu-baseline"; [ "$cfg" = 3full ] && { cfg=3; extra=""; }
      for i in $(seq $n); do
        f=$O/bench_cfg${cfg}_$i.json
        timeout -k 10 400 python -u bench.py --config $cfg $extra > $f 2> $O/bench_cfg${cfg}_$i.err || { tail -20 $O/bench_cfg${cfg}_$i.err; exit 1; }
        summ $f "cfg$cfg#$i" | tee -a $O/summary.txt
      done ;;
    ab)
      bash tools/ab_x3.sh ${val//:/ } > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
      grep -v amdgpu.ids $O/ab.txt ;;
    mlp)
      timeout -k 10 200 python -u tools/bench_mlp_train.py $AB_ARGS > $O/mlp.txt 2>&1 || { tail -20 $O/mlp.txt; exit 1; }
      grep -v amdgpu.ids $O/mlp.txt ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$val -o run -- python3 bench.py --config $val --no-cpu-baseline > $O/prof$val.log 2>&1 || { tail -20 $O/prof$val.log; exit 1; }
      head -12 $O/prof$val/run_kernel_stats.csv | cut -c1-160 ;;
    pmc)
      bash tools/gpu_pmc.sh $TAG/pmc$val $val || exit 1 ;;
    envsteps)  # val: "variant nb_car nb_ped nb_lines" with '_' for spaces, e.g. envsteps=4cars_4_1_2
      ROLLOUT_CFG="${val//_/ }" timeout -k 10 300 python -u tools/env_steps.py $O/envsteps_$val.json > $O/envsteps_$val.txt 2>&1 || { tail -20 $O/envsteps_$val.txt; exit 1; }
      tail -25 $O/envsteps_$val.txt ;;
    py)
      s=${val%%:*}; a=${val#*:}; [ "$a" = "$val" ] && a=""
      timeout -k 10 600 python -u tools/$s ${a//:/ } > $O/$s.txt 2>&1 || { tail -30 $O/$s.txt; exit 1; }
      tail -30 $O/$s.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done; done
exit 0
