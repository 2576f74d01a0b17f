#!/bin/bash
# Instruction attribution of the engine (run on the GPU box from the repo
# root): each build variants/valu/<name>.so (tools/build_variant.sh with
# -DCAIRO_TOOLS_BUILD -DCAIRO_ATTR_SKIP=<bit>; kernels.hip "Attribution
# builds") is copied over the in-tree library in turn and bench.py runs under
# one --pmc pass of the SQ instruction counters.  The drop of SQ_INSTS_VALU
# against the default build is what the skipped phase issues.  The in-tree
# library is put back however the runs end.
# COUNTERS overrides the counter list (e.g. the LDS counters, to attribute
# bank conflicts the same way).
# usage: [COUNTERS="..."] bash tools/attr_valu.sh [config] [build dir (default variants/valu)]
set -e
C=${1:-4k}
D=${2:-variants/valu}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/valu_$C${SFX:-}
rm -rf $OUT && mkdir -p $OUT
cp cairo_amd/_lib/libcairo_amd.so $OUT/.saved.so
trap 'cp $OUT/.saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
ARGS="--config $C --steps 6 --warmup 2 --no-verify --no-end-to-end --no-cpu-baseline --no-api --no-host-rgb"
for so in $D/*.so; do
  v=$(basename $so .so)
  cp $so cairo_amd/_lib/libcairo_amd.so
  timeout -k 10 300 rocprofv3 --pmc ${COUNTERS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE} --output-format csv -d $OUT/$v -o run -- python3 bench.py $ARGS > $OUT/$v.log 2>&1
  echo "$v done"
done
