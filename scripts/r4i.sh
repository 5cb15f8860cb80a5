# coarse approx A/B: parity tests touching the coarse ranking, then I1 / P1-shape phases
mkdir -p gpurun_out/r4i && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bench_configs.py tests/test_gpu_async.py tests/test_gpu_ivf.py tests/test_gpu_dims.py tests/test_gpu_pq.py > gpurun_out/r4i/tests.log 2>&1 || { tail -30 gpurun_out/r4i/tests.log; exit 1; }
tail -1 gpurun_out/r4i/tests.log
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_COARSE_APPROX=1,0,1 > gpurun_out/r4i/sweep.log 2>&1 || exit 1; tail -3 gpurun_out/r4i/sweep.log
