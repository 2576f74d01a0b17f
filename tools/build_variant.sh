#!/bin/bash
# Build a variant of libcairo_amd.so with extra kernel defines for A/B timing
# (tools/ab_bench.sh): scratch/ab/<name>.so.  The host objects come from the
# regular build (make first).
# usage: [KSRC=other_kernels.hip] bash tools/build_variant.sh <name> [-DFOO=1 ...]
set -e
N=$1; shift
mkdir -p scratch/ab build/obj/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -pthread -munsafe-fp-atomics "$@" \
  -I cairo_amd/csrc -c ${KSRC:-cairo_amd/csrc/kernels.hip} -o build/obj/ab/kernels_$N.o
OBJS=$(ls build/obj/*.o | grep -v '/kernels.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scratch/ab/$N.so build/obj/ab/kernels_$N.o $OBJS -lpthread
echo "built scratch/ab/$N.so"
