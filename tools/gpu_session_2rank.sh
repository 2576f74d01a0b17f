#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks on
# device 0 (CAIRO_BENCH_SHARED_DEVICE=1, gloo), the single-stream group leg and
# the replicas, every frame checked.
set -o pipefail
D=${1:-gpurun_out/r06_2rank}
mkdir -p $D
CAIRO_BENCH_SHARED_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 \
  --no-cpu-baseline --no-api --no-host-rgb > $D/bench_4k_2rank.json 2> $D/bench_4k_2rank.err
