#!/bin/bash
# Frames per launch at one frame size, alternating: bench.py --batch B.
# usage: bash tools/sweep_batch.sh <config> <rounds> <batch>...
set -e
C=$1; N=$2; shift 2
mkdir -p gpurun_out/sweep_batch
for i in $(seq 1 $N); do
  for b in "$@"; do
    timeout -k 10 300 python -u bench.py --config $C --batch $b --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb > gpurun_out/sweep_batch/${C}_${b}_${i}.log 2>&1
    echo "$C batch $b round $i $(tail -1 gpurun_out/sweep_batch/${C}_${b}_${i}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["engine_busy_ms_per_frame"], d["bit_exact"]["bit_exact"], d["bit_exact"]["frames_checked"])')"
  done
done
