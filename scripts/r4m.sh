#!/bin/bash
# Round-4 final measurement on the committed tree: smoke(), the default bench line, and the same bench under
# rocprofv3 --kernel-trace --stats (csv summaries only)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
find $O/kt -name "*kernel_trace.csv" -delete
tail -n 1 $O/bench_prof.log | cut -c1-200
