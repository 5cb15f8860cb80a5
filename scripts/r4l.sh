#!/bin/bash
# sprep split over SPREP_SPLIT blocks per item: the full GPU suite, the I1 sweep, and the kernel stats
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 20 PYR_COARSE_APPROX=1,1 > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
tail -n 2 $O/sweep.log | cut -c1-220
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 scripts/sweep_ivf.py --steps 10 > $O/sweep_prof.log 2>&1 || { tail -20 $O/sweep_prof.log; exit 1; }
find $O/kt -name "*kernel_trace.csv" -delete
grep -E "sprep|sample16|sselect|scan_kernel<128" $O/kt/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
