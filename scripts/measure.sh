#!/bin/bash
# One parametrized GPU-box measurement step (replaces round 4's one-off r4*.sh launchers).
#
#   bash scripts/measure.sh <outdir> <step> [args...]
#
# Steps (each under its own time limit; the exit status is the step's, so steps chain with &&):
#   tests <secs> [pytest args...]      the -m gpu suite (or the given test paths), verbose, per-test timeout
#   bench <name> <secs> [bench args]   python bench.py ... -> <outdir>/<name>.log; prints the JSON's headline
#   kt <name> <secs> [bench args]      the same under rocprofv3 --kernel-trace --stats (csv under <outdir>/<name>/)
#   pmc <name> <counters> [bench args] one rocprofv3 --pmc pass (its own run; counters of one block budget)
#   aux <name> <secs> <script> [args]  python -u <script> args -> <outdir>/<name>.log
#   ktaux <name> <secs> <script> [args]  the same under rocprofv3 --kernel-trace --stats (csv under <outdir>/<name>/)
#   pmcaux <name> <secs> <counters> <script> [args]  one rocprofv3 --pmc pass over a script
# P1 (IVF_PQ d=768 N=50M nlist=4096 m=96 nprobe=64, 10k queries; ~5 min of build):
#   bash scripts/measure.sh <outdir> aux p1 1100 scripts/bench_aux.py ivfpq --n 50000000 --train-rows 1048576 \
#        --nlist 4096 --m 96 --nprobe 64 --nq 10000 --steps 3 --check 2000 --recall-queries 200
#
# Example: bash scripts/measure.sh gpurun_out/r5a tests 300 && bash scripts/measure.sh gpurun_out/r5a bench i1 400
set -o pipefail
export TMPDIR=/tmp
export PYR_DEV_KNOBS=1  # A/B and measurement switches (kernels.h knob()); the driver's bench runs without
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=$1; step=$2; shift 2
mkdir -p "$O"

headline() {  # the bench JSON line's key figures
  grep '^{' "$1" | tail -n 1 | python3 -c "
import json, sys
try:
    d = json.loads(sys.stdin.read())
except ValueError:
    print('no JSON line'); sys.exit(0)
r = d.get('roofline') or {}
print(d.get('config', {}).get('workload'), 'n_gpus', d.get('n_gpus'), 'QPS %.0f' % d['value'], 'ms/step %.4f' % d['ms_per_step'],
      'recall', d.get('recall_at_10'), 'frac', r.get('frac'), 'phases', d.get('phases_ms'),
      'reruns', (d.get('exact_reruns') or {}).get('queries'))"
}

case "$step" in
  tests)
    secs=$1; shift
    [ $# -eq 0 ] && set -- -m gpu tests
    timeout -k 10 "$secs" python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > "$O/tests.log" 2>&1
    rc=$?
    grep -E "passed|failed|error" "$O/tests.log" | tail -n 3
    [ $rc -ne 0 ] && tail -n 40 "$O/tests.log"
    exit $rc ;;
  bench)
    name=$1; secs=$2; shift 2
    timeout -k 10 "$secs" python -u bench.py "$@" > "$O/$name.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { tail -n 30 "$O/$name.log"; exit $rc; }
    echo "$name: $(headline "$O/$name.log")" ;;
  kt)
    name=$1; secs=$2; shift 2
    timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- \
      python3 bench.py "$@" > "$O/$name.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { tail -n 30 "$O/$name.log"; exit $rc; }
    echo "$name: $(headline "$O/$name.log")" ;;
  pmc)
    name=$1; ctrs=$2; shift 2
    timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv -d "$O/$name" -o run -- python3 bench.py "$@" \
      > "$O/$name.log" 2>&1
    rc=$?
    [ $rc -ne 0 ] && { tail -n 30 "$O/$name.log"; exit $rc; }
    echo "$name: done" ;;
  aux)
    name=$1; secs=$2; script=$3; shift 3
    timeout -k 10 "$secs" python -u "$script" "$@" > "$O/$name.log" 2>&1
    rc=$?
    tail -n 12 "$O/$name.log"
    exit $rc ;;
  ktaux)
    name=$1; secs=$2; script=$3; shift 3
    timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$name" -o run -- \
      python3 -u "$script" "$@" > "$O/$name.log" 2>&1
    rc=$?
    tail -n 12 "$O/$name.log"
    exit $rc ;;
  pmcaux)
    name=$1; secs=$2; ctrs=$3; script=$4; shift 4
    timeout -s KILL "$secs" rocprofv3 --pmc $ctrs --output-format csv -d "$O/$name" -o run -- python3 -u "$script" "$@" \
      > "$O/$name.log" 2>&1
    rc=$?
    tail -n 6 "$O/$name.log"
    exit $rc ;;
  *)
    echo "unknown step $step" >&2; exit 2 ;;
esac
