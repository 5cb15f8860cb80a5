# full GPU suite + bench on the current tree
mkdir -p gpurun_out/r4f && export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r4f/tests.log 2>&1; rc=$?
tail -15 gpurun_out/r4f/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r4f/bench.json 2> gpurun_out/r4f/bench.log || exit 1; tail -1 gpurun_out/r4f/bench.json | cut -c1-400
