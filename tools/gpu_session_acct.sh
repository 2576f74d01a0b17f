#!/bin/bash
# One GPU call: accounting runs (tools/acct_run.sh) of variants/acct builds.
# usage: bash tools/gpu_session_acct.sh <out dir> "<name> <helpers>" ...
set -o pipefail
D=$1; shift
mkdir -p $D
for spec in "$@"; do
  read -r v h <<< "$spec"
  timeout -k 10 240 bash tools/acct_run.sh $v $D/acct_${v}_$h.json --helpers $h > $D/acct_${v}_$h.log 2>&1 || exit 1
done
