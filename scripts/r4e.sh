# attribution of the LDS sample kernel (ablation bits: 2048 no scoring, 4096 no tile loads, 1024 the
# one-wave-per-group sample_kernel); the kernel's own time from a kernel trace
mkdir -p gpurun_out/r4e && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/sweep_ivf.py --steps 10 PYR_FILTER_ABLATE=0,2048,4096,6144,1024 > gpurun_out/r4e/abl.log 2>&1 || exit 1; tail -5 gpurun_out/r4e/abl.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4e/kt -o run -- python3 scripts/sweep_ivf.py --steps 5 > gpurun_out/r4e/kt.log 2>&1 || exit 1
find gpurun_out/r4e/kt -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4e/kernel_stats.csv \;
find gpurun_out/r4e/kt -name "*.db" -delete; find gpurun_out/r4e/kt -name "*kernel_trace.csv" -delete
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r4e/kernel_stats.csv')):
    n=r['Name']
    if any(x in n for x in ('sample','sprep','stream16','sselect','scan_kernel','cand_merge','coarse','refine','ivf_')): print(n[:80], r['Calls'], r['AverageNs'])
"
