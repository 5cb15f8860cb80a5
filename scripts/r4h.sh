# I1 phases only
mkdir -p gpurun_out/r4h && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_SCAN_SAMPLE=0,0 > gpurun_out/r4h/sweep.log 2>&1 || exit 1; tail -2 gpurun_out/r4h/sweep.log
