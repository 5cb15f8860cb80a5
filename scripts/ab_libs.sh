#!/bin/bash
# A/B of prebuilt library variants on the I1 index (measurement only): for each name X given, the library
# pyrope_amd/ab_X.so (or the default build for "main") runs scripts/scan_ab.py in its own process, twice, in
# interleaved order.   bash scripts/ab_libs.sh <outdir> main A ...
set -o pipefail
O=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = main ]; then L=""; else L="pyrope_amd/ab_$v.so"; fi
    PYR_LIB=$L bash scripts/measure.sh "$O" aux "ab_${v}_$rep" 200 scripts/scan_ab.py --rounds 1 --reps 30 --variants "$v:" || exit 1
  done
done
