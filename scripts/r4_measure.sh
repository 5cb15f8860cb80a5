#!/bin/bash
# Round-4 measurement call on the GPU box: GPU tests, the bench (N=1), the list-scan sweep (round-4 vs
# round-3 kernels) and the rocprofv3 kernel-trace summary of the bench, each under its own time limit,
# chained so that a failure ends the call.  Logs under gpurun_out/r4/.
#   bash scripts/r4_measure.sh [steps...]   steps: diag tests bench sweep prof (default: all)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4
mkdir -p "$O"
steps=${*:-"diag tests bench sweep prof"}
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "[r4] $name: $*" >&2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[r4] $name rc=$rc" >&2
  tail -n 12 "$O/$name.log" >&2
  return $rc
}
for s in $steps; do
  case $s in
    diag) run diag 300 env PYR_STREAM_DEBUG=1 python -u scripts/diag/flat_cos_cert.py || exit $? ;;
    tests) run tests 600 python -u -m pytest -q --maxfail=25 --timeout 120 --timeout-method thread -m gpu tests/ || exit $? ;;
    bench) run bench 600 python -u bench.py || exit $? ;;
    sweep) run sweep 600 python -u scripts/sweep_ivf.py --steps 10 PYR_STREAM_MFMA=32,16 || exit $? ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 bench.py --steps 10 --cpu-seconds 0 --recall-queries 0 || exit $? ;;
    small) run small 600 python -u scripts/small_batch.py --sizes 1,64,256,1024 || exit $? ;;
  esac
done
