set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in "scalable 8 1 4" "4cars 4 1 2"; do
for r in 1 2; do
for p in 2 3 4 1; do
  MHPPO_ROLLOUT_PARTS=$p ROLLOUT_CFG="$cfg" timeout -k 10 200 python -u tools/bench_rollout.py > $O/p${p}_$r.txt 2>&1 || { tail -20 $O/p${p}_$r.txt; exit 1; }
  echo "$cfg parts=$p #$r $(grep 'iter 2' $O/p${p}_$r.txt | sed 's/policy rows.*//')" | tee -a $O/summary.txt
done; done; done
