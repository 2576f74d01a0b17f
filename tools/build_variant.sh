#!/bin/bash
# Build a variant of libcairo_amd.so with extra kernel defines for A/B timing
# (tools/ab_bench.sh): build/ab/<name>.so.  The host objects come from the
# regular build (make first).
# usage: bash tools/build_variant.sh <name> [-DFOO=1 ...]
set -e
N=$1; shift
mkdir -p build/ab build/obj/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -pthread -munsafe-fp-atomics "$@" \
  -c cairo_amd/csrc/kernels.hip -o build/obj/ab/kernels_$N.o
OBJS=$(ls build/obj/*.o | grep -v '/kernels.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ab/$N.so build/obj/ab/kernels_$N.o $OBJS -lpthread
echo "built build/ab/$N.so"
