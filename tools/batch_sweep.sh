#!/bin/bash
# Frames-per-launch sweep on the GPU box (run from the repo root):
#   bash tools/batch_sweep.sh <config> <rounds> <batch>...
# Alternates the batch sizes for <rounds> rounds; prints "batch round Mpix/s".
set -e
C=$1; N=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for b in "$@"; do
    timeout -k 10 200 python -u bench.py --config $C --no-cpu-baseline --no-end-to-end --batch $b > gpurun_out/bs_${C}_${b}_$i.log 2>&1
    echo "$C batch=$b round=$i $(tail -1 gpurun_out/bs_${C}_${b}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
