#!/bin/bash
# Run tools/acct.py on an accounting build (variants/acct/<name>.so, built with
# tools/build_variant.sh <name> -DCAIRO_ACCT=1) in place of the in-tree
# library, which is put back however the run ends (GPU box, repo root).
# usage: bash tools/acct_run.sh <name> <json out> [acct.py args...]
set -e
N=$1; J=$2; shift 2
mkdir -p gpurun_out
cp cairo_amd/_lib/libcairo_amd.so gpurun_out/.acct_saved.so
trap 'cp gpurun_out/.acct_saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
cp variants/acct/$N.so cairo_amd/_lib/libcairo_amd.so
python -u tools/acct.py --json "$J" "$@"
