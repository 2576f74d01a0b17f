#!/bin/bash
# Fabric-read attribution of the engine (run on the GPU box from the repo
# root): each diagnostic build scratch/attr/<name>.so (tools/build_variant.sh
# with -DCAIRO_TOOLS_BUILD -DCAIRO_ATTR_SKIP=..., kernels.hip) is copied over the in-tree library
# in turn and bench.py runs under ONE --pmc pass of sized read requests and
# write requests; tools/attr_summary.py then turns the per-build differences
# into bytes per frame.  The in-tree library is put back however the runs end.
# usage: bash tools/attr_traffic.sh [config] [build dir (default scratch/attr)]
set -e
C=${1:-4k}
D=${2:-scratch/attr}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/attr_$C$( [ "$D" = scratch/attr ] || echo _$(basename $D) )
rm -rf $OUT && mkdir -p $OUT
cp cairo_amd/_lib/libcairo_amd.so $OUT/.saved.so
trap 'cp $OUT/.saved.so cairo_amd/_lib/libcairo_amd.so' EXIT
ARGS="--config $C --no-end-to-end --no-cpu-baseline --no-api --no-host-rgb --steps 10"
for v in $(cd $D && ls *.so | sed 's/\.so$//'); do
  cp $D/$v.so cairo_amd/_lib/libcairo_amd.so
  echo "[attr] $v"
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum \
    --output-format csv -d $OUT/$v -o run -- python3 bench.py $ARGS > $OUT/$v.log 2>&1
done
echo "attributed: now run python tools/attr_summary.py --src $OUT locally"
