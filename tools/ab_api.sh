#!/bin/bash
# A/B of the synchronous drop-in API leg (bench.py api_encode: one frame per
# encode() call, latency-bound) for the builds in variants/ab/ (GPU box, repo
# root); the in-tree library is put back however the runs end.
# usage: bash tools/ab_api.sh <config> <rounds>
set -e
C=${1:-4k}; N=${2:-2}
mkdir -p gpurun_out
cp cairo_amd/_lib/libcairo_amd.so gpurun_out/.api_saved.so
trap 'cp gpurun_out/.api_saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
for i in $(seq 1 $N); do
  for v in $(cd variants/ab && ls *.so | sed 's/\.so$//'); do
    cp variants/ab/$v.so cairo_amd/_lib/libcairo_amd.so
    timeout -k 10 300 python -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-end-to-end --no-host-rgb --no-verify > gpurun_out/api_${C}_${v}_$i.log 2>&1
    echo "$v $i $(tail -1 gpurun_out/api_${C}_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["api_encode"]["fps"])')"
  done
done
