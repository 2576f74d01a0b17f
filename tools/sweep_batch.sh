#!/bin/bash
# Frames per launch at one frame size and a fixed number of timed frames,
# alternating: bench.py --batch B --steps FRAMES/B.
# usage: bash tools/sweep_batch.sh <config> <rounds> <timed frames> <batch>...
set -e
C=$1; N=$2; F=$3; shift 3
mkdir -p gpurun_out/sweep_batch
for i in $(seq 1 $N); do
  for b in "$@"; do
    log=gpurun_out/sweep_batch/${C}_${b}_${F}_${i}.log
    timeout -k 10 300 python -u bench.py --config $C --batch $b --steps $((F / b)) --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb > $log 2>&1
    echo "$C batch $b steps $((F / b)) round $i $(tail -1 $log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["engine_busy_ms_per_frame"], d["bit_exact"]["bit_exact"], d["bit_exact"]["frames_checked"])')"
  done
done
