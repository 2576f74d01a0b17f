#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit; an
# ordinary failure (exit 1: a failing test, a bench error) does not stop the
# session, but a fault, abort, segfault, kill or time limit (124, 134, 137,
# 139, or any status above 128) ends it: nothing more touches the GPU.
# usage: bash tools/gpu_steps.sh <outdir> "<seconds> <name> <command...>" ...
OUT=$1; shift
mkdir -p "$OUT"
for step in "$@"; do
  read -r secs name cmd <<< "$step"
  echo "[gpu_steps] $name: $cmd" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.out" 2> "$OUT/$name.err"
  rc=$?
  echo "[gpu_steps] $name exit $rc" | tee -a "$OUT/steps.log"
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then
    echo "[gpu_steps] stopping after $name (exit $rc)" | tee -a "$OUT/steps.log"
    exit $rc
  fi
done
