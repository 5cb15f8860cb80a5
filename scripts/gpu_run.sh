#!/bin/bash
# GPU-box helper: run one named measurement step with its own time limit, logging under gpurun_out/.
#   bash scripts/gpu_run.sh <name> <seconds> <command...>
# exits with the step's status, so steps chain with &&.
set -o pipefail
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "[gpu_run] $name: $*" >&2
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[gpu_run] $name rc=$rc" >&2
tail -n 40 "gpurun_out/$name.log" >&2
exit $rc
