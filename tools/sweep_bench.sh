#!/bin/bash
# One bench.py run per argument set (in-tree library), value printed per line.
# usage: bash tools/sweep_bench.sh <config> "<args 1>" "<args 2>" ...
set -e
C=$1; shift
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb $a > gpurun_out/sweep_${C}_$i.log 2>&1
  echo "[$a] $(tail -1 gpurun_out/sweep_${C}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["engine_busy_ms_per_frame"])')"
done
