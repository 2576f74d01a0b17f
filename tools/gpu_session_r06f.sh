#!/bin/bash
# GPU suite on the in-tree build, A/B of variants/ab, then the pool split around the default.
set -o pipefail
D=gpurun_out/r06f
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputest.txt 2>&1 &&
timeout -k 10 400 bash tools/ab_bench.sh 4k 3 > $D/ab.txt 2>&1 &&
timeout -k 10 400 bash tools/sweep_helpers.sh 1 $D "4k band4 200" "4k band4 208" "4k band4 216" "4k band4 224" "4k noise 200" "4k noise 216"
