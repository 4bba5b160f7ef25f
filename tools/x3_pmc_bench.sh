#!/bin/bash
# SQ counters of the training kernels inside bench.py (real rollout data), the same two counter
# passes as tools/x3_pmc.sh; usage (via gpurun): bash tools/x3_pmc_bench.sh <tag> [config]
set -o pipefail
OUT=gpurun_out/${1:-x3pmcb}; CFG=${2:-3}; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py --config $CFG --no-cpu-baseline --steps 1 --warmup 1 > $OUT/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -20 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_sq.py --kernel mlp_train_x3 $OUT/p1 $OUT/p2 > $OUT/summary.txt && cat $OUT/summary.txt
