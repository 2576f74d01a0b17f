#!/bin/bash
# Where a synchronous 4K encode() spends its time: kernel and copy trace of the
# drop-in C++ caller (8 frames), with the encoder's own per-frame split.
set -o pipefail
D=gpurun_out/r06m
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CAIRO_ENCODE_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $D/api -o run -- cairo_amd/_lib/evx1_api_caller 3840 2160 4 16 8 > $D/api.json 2> $D/api_trace.txt
