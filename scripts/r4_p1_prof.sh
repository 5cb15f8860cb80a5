#!/bin/bash
# P1 profiles (GPU box): rocprofv3 kernel stats of a timing run, then one counter pass over the IVF_PQ
# scan kernels (HBM bytes, MFMA busy); the large trace databases are summarized and removed.
set -o pipefail
export TMPDIR=/tmp PYR_PROGRESS=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r4_p1
mkdir -p $O
A="scripts/bench_aux.py ivfpq --n 50000000 --train-rows 1048576 --nlist 4096 --m 96 --nprobe 64 --nq 10000 --steps 3 --check 0"
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $A \
  > $O/kt.json 2> $O/kt.log || exit $?
find $O/kt -name "*kernel_trace.csv" -delete
cut -c1-400 $O/kt.json
timeout -s KILL 700 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "pq_scan_kernel|pq_prep_kernel|pq_refine_kernel" -d $O/pmc -o run -- python3 $A --steps 1 \
  > $O/pmc.json 2> $O/pmc.log || exit $?
python3 scripts/pmc_dispatch.py $O/pmc > $O/pmc.txt 2>&1
find $O/pmc -name "*.db" -delete
tail -6 $O/pmc.txt
