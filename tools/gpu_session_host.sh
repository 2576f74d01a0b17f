#!/bin/bash
# One GPU call: a bench line (hot path + host-RGB leg) of variants/ab/<name>.so,
# the in-tree library put back however it ends.
# usage: bash tools/gpu_session_host.sh <out dir> <name> [bench args...]
set -o pipefail
D=$1; V=$2; shift 2
mkdir -p $D
cp cairo_amd/_lib/libcairo_amd.so gpurun_out/.host_saved.so
trap 'cp gpurun_out/.host_saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
cp variants/ab/$V.so cairo_amd/_lib/libcairo_amd.so
timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $D/bench_$V.json 2> $D/bench_$V.err
