#!/bin/bash
# Rehearsal of the N > 1 bench step on a one-GPU box: 2 and 4 ranks on cuda:0 over gloo (PYR_BENCH_REHEARSE=1)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4n
mkdir -p $O
for n in 2 4; do
  PYR_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus $n --steps 20 > $O/rehearse_$n.log 2>&1 || { tail -30 $O/rehearse_$n.log; exit 1; }
  tail -n 1 $O/rehearse_$n.log | cut -c1-300
done
