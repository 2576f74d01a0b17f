#!/bin/bash
# The round-end checks the driver runs, on the in-tree build: GPU suite, smoke, default bench line.
set -o pipefail
D=${1:-gpurun_out/check}
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputest.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.txt 2>&1 &&
timeout -k 10 300 python -u bench.py > $D/bench.json 2> $D/bench.err
