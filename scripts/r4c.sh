# round-4 sample-in-LDS check: parity on the stream paths, then A/B against the round-3 sample
mkdir -p gpurun_out/r4c && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dims.py tests/test_gpu_ivf.py tests/test_gpu_bench_configs.py tests/test_gpu_flat.py tests/test_gpu_cosine.py tests/test_gpu_certificate.py > gpurun_out/r4c/tests.log 2>&1 || { tail -30 gpurun_out/r4c/tests.log; exit 1; }
tail -2 gpurun_out/r4c/tests.log
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_SCAN_SAMPLE=0,3 PYR_FILTER_ABLATE=0,1024 > gpurun_out/r4c/sample.log 2>&1 || exit 1; tail -6 gpurun_out/r4c/sample.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4c/bench.json 2> gpurun_out/r4c/bench.log || exit 1; tail -1 gpurun_out/r4c/bench.json | cut -c1-900
