#!/bin/bash
# A/B timing of library builds at several pool splits on the GPU box (run from
# the repo root): per round, each "variant helpers" spec copies
# variants/ab/<variant>.so over the in-tree library and runs bench.py with
# --helpers (0 = the build's default), alternating, $2 rounds.
# usage: bash tools/ab_sweep.sh <config> <rounds> "A 0" "B 0" "B 184" ...
set -e
C=$1; N=$2; shift 2
mkdir -p gpurun_out
cp cairo_amd/_lib/libcairo_amd.so gpurun_out/.ab_saved.so
trap 'cp gpurun_out/.ab_saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
for i in $(seq 1 $N); do
  for spec in "$@"; do
    read -r v h <<< "$spec"
    cp variants/ab/$v.so cairo_amd/_lib/libcairo_amd.so
    L=gpurun_out/abs_${C}_${v}_${h}_$i.log
    timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb --helpers $h > $L 2>&1
    echo "$v $h $i $(tail -1 $L | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["bit_exact"])')"
  done
done
