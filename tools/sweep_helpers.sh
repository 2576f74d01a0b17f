#!/bin/bash
# Helper/coder pool split sweep on the GPU box (run from the repo root):
# bench.py per "config content helpers" spec, $1 rounds, values appended to
# $2/sweep.txt.
# usage: bash tools/sweep_helpers.sh <rounds> <outdir> "4k band4 192" "4k band4 200" ...
set -e
N=$1; O=$2; shift 2
mkdir -p $O
for r in $(seq 1 $N); do
  for spec in "$@"; do
    read -r c t h <<< "$spec"
    timeout -k 10 300 python -u bench.py --config $c --content $t --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb --helpers $h > $O/${c}_${t}_$h.$r.log 2>&1
    echo "$spec $r $(tail -1 $O/${c}_${t}_$h.$r.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')" >> $O/sweep.txt
  done
done
