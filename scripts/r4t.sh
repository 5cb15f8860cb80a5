#!/bin/bash
# Sample pass in half-item units (two 8-wave blocks per CU) vs one item per block (HEAD's library):
# the GPU suite, then alternating I1 sweeps
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for i in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export PYR_LIB=$PWD/pyrope_amd/libpyrope_hip_head.so; else unset PYR_LIB; fi
    timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 20 > $O/sweep_${v}_$i.log 2>&1 || { tail -20 $O/sweep_${v}_$i.log; exit 1; }
    echo "$v $i: $(tail -n 1 $O/sweep_${v}_$i.log | cut -c1-200)"
  done
done
