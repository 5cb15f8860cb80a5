#!/bin/bash
# P1 (IVF_PQ d=768 N=50M nlist=4096 m=96 nprobe=64, 10k queries) at full size on the GPU box: timing,
# a 2,000-query oracle parity sample, recall@10 vs exact FLAT (streamed), the LUT scan for A/B.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r4_p1
PYR_PROGRESS=1 timeout -k 10 1100 python -u scripts/bench_aux.py ivfpq --n 50000000 --train-rows 1048576 --nlist 4096 --m 96 \
  --nprobe 64 --nq 10000 --steps 3 --check ${P1_CHECK:-2000} --recall-queries ${P1_RECALL:-200} --sweep "${P1_SWEEP:-PYR_PQ_MFMA=0}" \
  > gpurun_out/r4_p1/p1.json 2> gpurun_out/r4_p1/p1.log
rc=$?
tail -4 gpurun_out/r4_p1/p1.log
cut -c1-1500 gpurun_out/r4_p1/p1.json
exit $rc
