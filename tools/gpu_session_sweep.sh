#!/bin/bash
# One GPU call: the GPU suite on the in-tree build (unless SKIP_TESTS), then
# tools/ab_sweep.sh over variants/ab at the given "variant helpers" specs.
# usage: [SKIP_TESTS=1] bash tools/gpu_session_sweep.sh <out dir> <config> <rounds> "A 0" "B 0" ...
set -o pipefail
D=$1; C=$2; N=$3; shift 3
mkdir -p $D
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputest.txt 2>&1; } &&
timeout -k 10 1000 bash tools/ab_sweep.sh $C $N "$@" > $D/sweep.txt 2>&1
