#!/bin/bash
# SQ counters of the env-step kernel (issue / wait / instruction mix / instruction cache), one
# rocprofv3 --pmc pass per counter group over tools/bench_rollout.py (65 536 4cars envs),
# summarised by tools/pmc_sq.py.  Usage (via gpurun, from the repo root): bash tools/env_pmc.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-envpmc}; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH"
P3="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVE_CYCLES"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/bench_rollout.py > $OUT/p$i.log 2>&1 || { echo "PMC pass $i FAILED"; tail -20 $OUT/p$i.log; break; }
done
python3 tools/pmc_sq.py --kernel sample_env $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/summary.txt; cat $OUT/summary.txt
