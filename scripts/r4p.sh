#!/bin/bash
# Sample tiles scaled to short lists (samp_div = 8, IVF path): the GPU suite, then one rank's step at the
# N = 4 / N = 8 rows-within-list shapes (lists of 76 / 38 tiles) in one process, HEAD's library vs this
# tree's, and the N = 4 rehearsal (4 ranks on cuda:0 over gloo) for the end-to-end result
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
for shape in "2500000 40000" "1250000 80000"; do
  set -- $shape
  for v in head new; do
    if [ $v = head ]; then export PYR_LIB=$PWD/pyrope_amd/libpyrope_hip_head.so; else unset PYR_LIB; fi
    timeout -k 10 300 python -u bench.py --n $1 --train-rows $1 --nq $2 --steps 20 --cpu-seconds 0 --recall-queries 0 > $O/rank_${1}_${v}.log 2>&1 || { tail -20 $O/rank_${1}_${v}.log; exit 1; }
    echo "n=$1 nq=$2 $v: $(tail -n 1 $O/rank_${1}_${v}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), d['phases_ms'], d['exact_reruns'].get('queries'))")"
  done
done
unset PYR_LIB
PYR_BENCH_REHEARSE=1 timeout -k 10 400 python -u bench.py --gpus 4 --steps 20 > $O/rehearse_4.log 2>&1 || { tail -30 $O/rehearse_4.log; exit 1; }
tail -n 1 $O/rehearse_4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['backend'], d['recall_at_10'], d['phases_ms'])"
