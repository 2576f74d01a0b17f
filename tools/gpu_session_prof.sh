#!/bin/bash
# Final-build profiles: rocprofv3 kernel trace + PMC passes of bench.py's 4K
# hot path (tools/profile_round.sh), then the time accounting build.
set -o pipefail
timeout -k 10 1000 bash tools/profile_round.sh r06 4k > gpurun_out/prof4k_r06.log 2>&1 &&
mkdir -p gpurun_out/r06n &&
timeout -k 10 200 bash tools/acct_run.sh acct_final gpurun_out/r06n/acct_final.json --steps 10 > gpurun_out/r06n/acct.log 2>&1
