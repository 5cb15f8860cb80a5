#!/bin/bash
# Final round-4 measurements (GPU box): the bench under rocprofv3 --kernel-trace --stats (csv summaries
# only), and the I1 list scan at d = 96 vs d = 128 (per-byte rate of the padded tile dimension).
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py \
  > $O/bench_prof.log 2>&1 || exit $?
find $O/kt -name "*kernel_trace.csv" -delete
tail -1 $O/bench_prof.log | cut -c1-300
for d in 96 128; do
  timeout -k 10 300 python -u scripts/sweep_ivf.py --dim $d --steps 10 > $O/dim$d.log 2>&1 || exit $?
  tail -2 $O/dim$d.log
done
