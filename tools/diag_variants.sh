#!/bin/bash
# Run a few parity tests against each library variant in scratch/diag (copied
# over the in-tree library in turn), one pytest process per variant.
# usage: bash tools/diag_variants.sh <outdir> <test node id> ...
OUT=$1; shift
mkdir -p $OUT
cp cairo_amd/_lib/libcairo_amd.so $OUT/orig.so
for v in $(cd scratch/diag && ls *.so | sed 's/\.so$//'); do
  cp scratch/diag/$v.so cairo_amd/_lib/libcairo_amd.so
  timeout -k 10 240 python -u -m pytest -q --tb=short --timeout 120 --timeout-method thread "$@" > $OUT/$v.txt 2>&1
  rc=$?
  echo "$v exit $rc: $(tail -1 $OUT/$v.txt)"
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "stopping"; break; fi
done
cp $OUT/orig.so cairo_amd/_lib/libcairo_amd.so
