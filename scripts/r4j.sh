#!/bin/bash
# Re-entry check on HEAD: the full GPU suite, smoke(), the default bench line and its rocprofv3 kernel stats.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --graph 0 > $O/bench_nograph.log 2>&1 || { tail -20 $O/bench_nograph.log; exit 1; }
tail -n 1 $O/bench_nograph.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 100 > $O/bench_100.log 2>&1 || { tail -20 $O/bench_100.log; exit 1; }
tail -n 1 $O/bench_100.log | cut -c1-200
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_COARSE_APPROX=1,1 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
tail -n 2 $O/sweep.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
find $O/kt -name "*kernel_trace.csv" -delete
tail -n 1 $O/bench_prof.log | cut -c1-200
