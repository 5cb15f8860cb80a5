# full GPU suite, I1 phases, bench
mkdir -p gpurun_out/r4g && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -q -x --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r4g/tests.log 2>&1; rc=$?
tail -15 gpurun_out/r4g/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_SCAN_SAMPLE=0,0 > gpurun_out/r4g/sweep.log 2>&1 || exit 1; tail -2 gpurun_out/r4g/sweep.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4g/bench.json 2> gpurun_out/r4g/bench.log || exit 1; tail -1 gpurun_out/r4g/bench.json | cut -c1-300
