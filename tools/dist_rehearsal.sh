#!/bin/bash
# Two bench ranks on the one GPU of a gpurun box (the multi-rank product path, not a scaling figure):
# gloo first, then RCCL (which may refuse two ranks on one device).  Output under gpurun_out/<tag>/.
set -o pipefail
O=gpurun_out/${1:-dist}; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for be in gloo nccl; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --dist-backend $be \
    > $O/bench2_$be.json 2> $O/bench2_$be.err
  rc=$?
  echo "backend $be rc $rc"; tail -c 700 $O/bench2_$be.json; echo; grep -i -m5 "error\|duplicate\|invalid" $O/bench2_$be.err
  [ $rc -ne 0 ] && break
done
exit 0
