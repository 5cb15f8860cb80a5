mkdir -p gpurun_out/r4 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_async.py tests/test_gpu_filter.py > gpurun_out/r4/t_async.log 2>&1; tail -3 gpurun_out/r4/t_async.log
timeout -k 10 400 python -u scripts/sweep_ivf.py --steps 10 PYR_STREAM_RMIN=8,4,2 PYR_STREAM_ET=8,4 > gpurun_out/r4/rank.log 2>&1 || exit 1; tail -7 gpurun_out/r4/rank.log
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_FILTER_ABLATE=0,512 > gpurun_out/r4/pf.log 2>&1 || exit 1; tail -3 gpurun_out/r4/pf.log
PYR_FILTER_ABLATE=512 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex scan_kernel -d gpurun_out/r4/fetch512 -o run -- python3 scripts/sweep_ivf.py --steps 3 > gpurun_out/r4/fetch512.log 2>&1 || exit 1
python scripts/pmc_dispatch.py gpurun_out/r4/fetch512 scan_kernel | tail -3
for m in 0 1 2; do timeout -k 10 300 python -u scripts/bench_aux.py flat --metric $m --steps 5 > gpurun_out/r4/f2_m$m.json 2> gpurun_out/r4/f2_m$m.log || exit 1; tail -1 gpurun_out/r4/f2_m$m.json | cut -c1-300; done
