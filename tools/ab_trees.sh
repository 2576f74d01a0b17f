#!/bin/bash
# A/B timing of two whole trees on the GPU box (run from the repo root): this
# tree ("new") and abtree/ ("old": a git worktree of another commit, built in
# place with make), alternating, $2 rounds.  NEW_ARGS: extra bench.py
# arguments for this tree only (e.g. --no-verify, which the old bench lacks).
# usage: bash tools/ab_trees.sh <config> <rounds> [bench args...]
set -e
C=${1:-4k}; N=${2:-2}; shift 2 || true
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in new old; do
    d=.; extra="$NEW_ARGS"
    if [ $v = old ]; then d=abtree; extra=""; fi
    (cd $d && timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-end-to-end --no-api \
      --no-host-rgb $extra "$@") > gpurun_out/abt_${C}_${v}_$i.log 2>&1
    echo "$v $i $(tail -n 1 gpurun_out/abt_${C}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["engine_busy_ms_per_frame"])')"
  done
done
