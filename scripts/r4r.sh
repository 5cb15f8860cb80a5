#!/bin/bash
# M8's shape on one GPU (IVF_FLAT d=128 N=80M nlist=8192 nprobe=32) on the round-4 kernels
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 900 python -u bench.py --n 80000000 --nlist 8192 --steps 20 --cpu-seconds 0 > $O/m8_1gpu.log 2>&1 || { tail -30 $O/m8_1gpu.log; exit 1; }
tail -n 1 $O/m8_1gpu.log | cut -c1-300
