#!/bin/bash
# One rank's N = 2 workload in one process (5M rows, 20,000 queries a step), phases and kernel stats: is the
# rehearsal's merge / sample time its own or the other rank's kernels sharing the GPU?
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --n 5000000 --train-rows 5000000 --nq 20000 --steps 20 --cpu-seconds 0 --recall-queries 0 > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
find $O/kt -name "*kernel_trace.csv" -delete
tail -n 1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['phases_ms'])"
grep -E "cand_merge|sample16|sprep|sselect|scan_kernel<128|refine_kernel" $O/kt/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
