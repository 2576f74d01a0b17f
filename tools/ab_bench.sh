#!/bin/bash
# A/B timing of builds of the library on the GPU box (run from the repo
# root): variants/ab/<variant>.so (A, B, ...) are copied in turn over the in-tree
# library and bench.py runs on each, alternating, $2 rounds.
# usage: bash tools/ab_bench.sh <config> <rounds> [bench args...]
set -e
C=${1:-720p}; N=${2:-2}; shift 2 || true
mkdir -p gpurun_out
# the in-tree library is put back however the runs end
cp cairo_amd/_lib/libcairo_amd.so gpurun_out/.ab_saved.so
trap 'cp gpurun_out/.ab_saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
for i in $(seq 1 $N); do
  for v in $(cd variants/ab && ls *.so | sed 's/\.so$//'); do
    cp variants/ab/$v.so cairo_amd/_lib/libcairo_amd.so
    timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb "$@" > gpurun_out/ab_${C}_${v}_$i.log 2>&1
    echo "$v $i $(tail -1 gpurun_out/ab_${C}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
