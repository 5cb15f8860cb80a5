set -o pipefail
for rep in 1 2; do
  for v in main r5; do
    if [ $v = main ]; then L=""; else L="pyrope_amd/ab_$v.so"; fi
    PYR_LIB=$L bash scripts/measure.sh gpurun_out/r6f2ab aux f2_${v}_$rep 200 scripts/bench_aux.py flat --n 1000000 --dim 128 --metric 0 --steps 10 --check 5 || exit 1
  done
done
