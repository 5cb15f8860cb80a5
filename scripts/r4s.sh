#!/bin/bash
# The driver's N > 1 launch (torch.distributed.run, one process per rank) rehearsed on one GPU:
# 2 ranks on cuda:0 over gloo (PYR_BENCH_REHEARSE=1)
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4s
mkdir -p $O
PYR_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 > $O/launcher_2.log 2>&1 || { tail -30 $O/launcher_2.log; exit 1; }
grep '^{"metric"' $O/launcher_2.log | cut -c1-300
