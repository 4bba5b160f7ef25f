#!/bin/bash
# SQ counters of the MFMA policy kernel over tools/bench_rollout.py (65 536 4cars envs), one
# rocprofv3 --pmc pass per group.  Usage (via gpurun, from the repo root): bash tools/policy_pmc.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-polpmc}; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/bench_rollout.py > $OUT/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -20 $OUT/p$i.log; break; }
done
python3 tools/pmc_sq.py --kernel policy $OUT/p1 $OUT/p2 > $OUT/summary.txt; cat $OUT/summary.txt
