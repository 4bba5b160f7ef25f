set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-iter}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
MHPPO_LIB=build_ab/timing/libmhppo.so timeout -k 10 120 python tools/env_phases.py 4cars 4 1 2 65536 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH FAILED; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo PROF FAILED; tail -30 $OUT/prof.err; exit 1; }
