#!/bin/bash
# One GPU call: the GPU suite on the in-tree build, then an A/B of the
# variants in variants/ab (tools/ab_bench.sh), then one SQ counter pass of
# the in-tree build; with K2=1 also the inter-frame lag at 4K (tools/k2_phases.py:
# a nearly idle GPU, 4 frames, and a loaded one, 32).  Every step has its own
# time limit and the steps are chained: the first failure ends the call.
# usage: [SKIP_TESTS=1] [K2=1] bash tools/gpu_session_ab.sh <out dir> [rounds] [config]
set -o pipefail
D=$1; N=${2:-3}; C=${3:-4k}
mkdir -p $D
ROOT=$(pwd)
{ [ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $D/gputest.txt 2>&1; } &&
{ [ "$N" = 0 ] || timeout -k 10 600 bash tools/ab_bench.sh $C $N > $D/ab.txt 2>&1; } &&
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" &&
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $D/prof_sq -o run -- python3 bench.py --config $C --no-verify --no-end-to-end --no-cpu-baseline --no-api --no-host-rgb > $D/prof_sq.log 2>&1 &&
{ [ -z "$K2" ] || { timeout -k 10 120 python -u tools/k2_phases.py --config 4k --batch 4 > $D/k2_4k_b4.txt 2>&1 &&
                    timeout -k 10 180 python -u tools/k2_phases.py --config 4k --batch 32 > $D/k2_4k_b32.txt 2>&1; }; }
