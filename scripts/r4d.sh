# sample A/B after a sample-kernel change: parity on the stream paths, then timings
mkdir -p gpurun_out/r4d && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dims.py tests/test_gpu_ivf.py tests/test_gpu_bench_configs.py tests/test_gpu_certificate.py > gpurun_out/r4d/tests.log 2>&1 || { tail -30 gpurun_out/r4d/tests.log; exit 1; }
tail -1 gpurun_out/r4d/tests.log
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_SCAN_SAMPLE=0,3,0 > gpurun_out/r4d/sample.log 2>&1 || exit 1; tail -3 gpurun_out/r4d/sample.log
