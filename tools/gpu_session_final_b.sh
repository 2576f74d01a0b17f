#!/bin/bash
# Round-end lines on the final build (2/2): 720p, 4K noise and static lines, the 4K quality sweep.
set -o pipefail
D=gpurun_out/final
mkdir -p $D
timeout -k 10 300 python -u bench.py --config 720p --intervals $D/intervals_720p_final.csv > $D/bench_720p_final.json 2> $D/bench_720p_final.err &&
timeout -k 10 300 python -u bench.py --content noise --intervals $D/intervals_4k_noise_final.csv > $D/bench_4k_noise_final.json 2> $D/bench_4k_noise_final.err &&
timeout -k 10 300 python -u bench.py --content static --intervals $D/intervals_4k_static_final.csv > $D/bench_4k_static_final.json 2> $D/bench_4k_static_final.err &&
timeout -k 10 400 python -u tools/rd_sweep.py --frames 240 --out $D/rd_sweep.json > $D/rd.log 2>&1
