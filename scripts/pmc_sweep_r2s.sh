cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r2s && \
S="scripts/sweep_ivf.py --steps 1 PYR_FILTER_PREC=2 PYR_FILTER_ABLATE=0,128" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex mfma_filter16 -d gpurun_out/r2s/fetch -o run -- python $S > gpurun_out/r2s/fetch.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex mfma_filter16 -d gpurun_out/r2s/sq -o run -- python $S > gpurun_out/r2s/sq.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex mfma_filter16 -d gpurun_out/r2s/mfma -o run -- python $S > gpurun_out/r2s/mfma.log 2>&1 && \
for p in fetch sq mfma; do python scripts/pmc_dispatch.py gpurun_out/r2s/$p mfma_filter16 > gpurun_out/r2s/$p.txt; done
