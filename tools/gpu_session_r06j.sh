#!/bin/bash
# GPU suite on the in-tree build (precode beside the engine), A/B of the
# precode placements, then one full bench line of the in-tree build.
set -o pipefail
D=gpurun_out/r06j
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputest.txt 2>&1 &&
timeout -k 10 500 bash tools/ab_bench.sh 4k 2 > $D/ab.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > $D/bench_full.json 2> $D/bench_full.err
