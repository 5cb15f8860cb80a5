#!/bin/bash
# Profile the bench workload on one MI355X (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats of `bench.py` (per-kernel durations; rocpd db + csv)
#   2. a FETCH_SIZE pass (HBM read bytes) restricted to the scan kernels
#   3. an SQ pass (VALU / LDS instruction mix, wave cycles) restricted to the scan kernels
#   4. an MFMA pass (MFMA instructions, MFMA busy cycles, GRBM_GUI_ACTIVE)
# Counter passes run alone (no --sys-trace etc.), each under its own kill timeout.
# Usage: scripts/profile.sh <tag> [extra bench.py args...]
set -u
TAG=${1:-r1}
shift || true
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$P"
cd "$ROOT" || exit 1
REGEX=${PYR_PROF_REGEX:-scan_|mfma_filter}
B="--cpu-seconds 0 --recall-queries 0"

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d "$P/kt" -o run -- \
  python bench.py --steps 10 --warmup 2 $B "$@" > "$P/kt_bench.json" 2> "$P/kt_bench.log" || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d "$P/fetch" -o run -- \
  python bench.py --steps 2 --warmup 1 --profile-steps 0 $B "$@" > "$P/fetch_bench.json" 2> "$P/fetch_bench.log" || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --kernel-include-regex "$REGEX" -d "$P/sq" -o run -- \
  python bench.py --steps 2 --warmup 1 --profile-steps 0 $B "$@" > "$P/sq_bench.json" 2> "$P/sq_bench.log" || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "$REGEX" -d "$P/mfma" -o run -- \
  python bench.py --steps 2 --warmup 1 --profile-steps 0 $B "$@" > "$P/mfma_bench.json" 2> "$P/mfma_bench.log" || exit $?
find "$P" -maxdepth 3 | head -60
