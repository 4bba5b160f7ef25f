#!/bin/bash
# One GRBM_GUI_ACTIVE pass over a short cfg3 bench, then the per-launch clock sequence of the train passes.
set -o pipefail
O=gpurun_out/${1:-clkseq}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/clk -o run -- python3 bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > $O/clk.log 2>&1 || { tail -20 $O/clk.log; exit 1; }
python3 tools/clock_sequence.py $O/clk/run_counter_collection.csv | tee $O/clock_sequence.txt
