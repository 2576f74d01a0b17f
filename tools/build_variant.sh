#!/bin/bash
# Build a variant of libcairo_amd.so with extra kernel defines for A/B timing
# (tools/ab_bench.sh, tools/attr_valu.sh): $VDIR/<name>.so (default
# variants/ab; variants/ is git-ignored but travels to the GPU box).  The host objects come from the
# regular build (make first); with HOSTDEFS=1 the backend (task order, launch
# sizing) is rebuilt with the same defines.
# usage: [KSRC=other_kernels.hip] [HOSTDEFS=1] bash tools/build_variant.sh <name> [-DFOO=1 ...]
set -e
N=$1; shift
V=${VDIR:-variants/ab}
mkdir -p $V build/obj/ab
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -pthread -munsafe-fp-atomics"
$HIPCC "$@" -I cairo_amd/csrc -c ${KSRC:-cairo_amd/csrc/kernels.hip} -o build/obj/ab/kernels_$N.o
EXCL='/kernels.o$'
EXTRA=""
if [ -n "$HOSTDEFS" ]; then
  $HIPCC "$@" -I cairo_amd/csrc -c cairo_amd/csrc/backend.hip -o build/obj/ab/backend_$N.o
  EXCL='/(kernels|backend).o$'
  EXTRA=build/obj/ab/backend_$N.o
fi
OBJS=$(ls build/obj/*.o | grep -Ev "$EXCL")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $V/$N.so build/obj/ab/kernels_$N.o $EXTRA $OBJS -lpthread
echo "built $V/$N.so"
