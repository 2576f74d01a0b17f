#!/bin/bash
# A/B of one environment switch of the in-tree library (GPU box, repo root):
# bench.py alternately without and with NAME=VALUE, $3 rounds.
# usage: bash tools/ab_env.sh <config> NAME=VALUE <rounds> [bench args...]
set -e
C=$1; KV=$2; N=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in off on; do
    if [ $v = on ]; then E="env $KV"; else E=""; fi
    $E timeout -k 10 400 python -u bench.py --config $C "$@" > gpurun_out/abenv_${C}_${v}_$i.log 2>&1
    echo "$v $i $(tail -1 gpurun_out/abenv_${C}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d.get("end_to_end") or {}; print(d["value"], e.get("value"), d["roofline"]["engine_busy_ms_per_frame"])')"
  done
done
