set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1 MHPPO_ROLLOUT_PARTS=1
O=gpurun_out/${1:-r06p}; mkdir -p $O
for cfg in "4cars 4 1 2" "scalable 8 1 4"; do
  t=${cfg// /_}
  ROLLOUT_CFG="$cfg" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 tools/bench_rollout.py > $O/prof_$t.log 2>&1 || { tail -20 $O/prof_$t.log; exit 1; }
  grep -v amdgpu.ids $O/prof_$t.log
  head -6 $O/prof_$t/run_kernel_stats.csv | cut -c1-150
done
ROLLOUT_CFG="scalable 8 1 4" bash tools/policy_pmc.sh ${1:-r06p}/pmc4 || exit 1
ROLLOUT_CFG="4cars 4 1 2" bash tools/policy_pmc.sh ${1:-r06p}/pmc3 || exit 1
