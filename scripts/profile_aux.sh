#!/bin/bash
# Profile a scripts/bench_aux.py workload on one MI355X (run on the GPU box via gpurun):
#   kernel trace + stats, then an SQ counter pass (VALU / LDS instruction mix, LDS bank
#   conflicts, wave cycles) and a FETCH_SIZE pass restricted to the kernels matching REGEX.
# Usage: scripts/profile_aux.sh <tag> <regex> <bench_aux args...>
set -u
TAG=$1; REGEX=$2; shift 2
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$P"
cd "$ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d "$P/kt" -o run -- \
  python scripts/bench_aux.py "$@" > "$P/kt.json" 2> "$P/kt.log" || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" -d "$P/sq" -o run -- \
  python scripts/bench_aux.py "$@" > "$P/sq.json" 2> "$P/sq.log" || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d "$P/fetch" -o run -- \
  python scripts/bench_aux.py "$@" > "$P/fetch.json" 2> "$P/fetch.log" || exit $?
ls "$P"
