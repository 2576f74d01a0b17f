#!/bin/bash
# Round-end lines on the final build (1/2): GPU suite, smoke, 4K and 1080p bench lines.
set -o pipefail
D=gpurun_out/final
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputest_final.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke_final.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --intervals $D/intervals_4k_final.csv > $D/bench_4k_final.json 2> $D/bench_4k_final.err &&
timeout -k 10 300 python -u bench.py --config 1080p --intervals $D/intervals_1080p_final.csv > $D/bench_1080p_final.json 2> $D/bench_1080p_final.err
