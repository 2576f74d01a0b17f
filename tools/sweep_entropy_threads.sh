#!/bin/bash
# End-to-end leg of bench.py at several host entropy thread counts, alternating,
# $2 rounds (GPU box, repo root).  usage: bash tools/sweep_entropy_threads.sh <out dir> <rounds> 14 15 16
set -o pipefail
D=$1; N=$2; shift 2
mkdir -p $D
for i in $(seq 1 $N); do
  for t in "$@"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api --no-host-rgb --no-verify --entropy-threads $t > $D/e2e_${t}_$i.json 2> $D/e2e_${t}_$i.err || exit 1
    echo "$t $i $(tail -1 $D/e2e_${t}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["end_to_end"]; print(d["value"], e["value"], e.get("steady_value"), e["pipeline"]["entropy_ms_per_frame_per_thread"])')" >> $D/sweep.txt
  done
done
