#!/bin/bash
# FETCH_SIZE of the engine per variant (scratch/ab/<variant>.so, as
# tools/ab_bench.sh): one rocprofv3 --pmc pass each over a short bench run;
# prints the median KiB per engine dispatch (after the first) and per frame.
# usage: bash tools/ab_fetch.sh <config> [counter]
set -e
C=${1:-4k}; K=${2:-FETCH_SIZE}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in $(cd scratch/ab && ls *.so | sed 's/\.so$//'); do
  cp scratch/ab/$v.so cairo_amd/_lib/libcairo_amd.so
  rm -rf gpurun_out/abf_$v
  timeout -s KILL 120 rocprofv3 --pmc $K --output-format csv -d gpurun_out/abf_$v -o run -- python3 bench.py --config $C --steps 6 --warmup 2 --no-cpu-baseline --no-end-to-end --no-api --no-host-rgb > gpurun_out/abf_$v.log 2>&1
  python3 - "$v" "$K" <<'PY'
import csv, glob, statistics, sys
v, k = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/abf_{v}/**/run_counter_collection.csv", recursive=True)[0]
vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_engine" in r["Kernel_Name"] and r["Counter_Name"] == k]
m = statistics.median(vals[1:])
print(v, k, "median KiB/dispatch", round(m), "dispatches", len(vals))
PY
done
