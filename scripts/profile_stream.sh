#!/bin/bash
# Counter passes over the IVF stream-and-emit list scan at the I1 config (run on the GPU box):
#   sweep   timing of the knob settings given as arguments (scripts/sweep_ivf.py)
#   sq      wave-state buckets (SQ_WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY), LDS stalls
#   mfma    MFMA instructions / busy cycles, GRBM_GUI_ACTIVE (clock), LDS bank conflicts
#   fetch   FETCH_SIZE (HBM read bytes; x2 on gfx950, MI355X_MICROARCH.md)
# Each counter pass runs alone under its own kill timeout.
# Usage: scripts/profile_stream.sh <tag> [sweep knobs...]
set -u
TAG=${1:-r3}
shift || true
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
P=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$P"
cd "$ROOT" || exit 1
REGEX=${PYR_PROF_REGEX:-scan_kernel}
S="python scripts/sweep_ivf.py --steps 3"

timeout -k 10 240 $S "$@" > "$P/sweep.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-include-regex "$REGEX" -d "$P/sq" -o run -- \
  $S > "$P/sq.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT \
  SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "$REGEX" -d "$P/mfma" -o run -- \
  $S > "$P/mfma.log" 2>&1 || exit $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$REGEX" -d "$P/fetch" -o run -- \
  $S > "$P/fetch.log" 2>&1 || exit $?
for d in sq mfma fetch; do python scripts/pmc_dispatch.py "$P/$d" > "$P/$d.txt" 2>&1; done
tail -n 4 "$P"/*.txt
