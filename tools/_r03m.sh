set -o pipefail
mkdir -p gpurun_out/r03m
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $R/gpurun_out/r03m/mfma -o run --output-format csv -- python3 $R/bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline --no-overlap > $R/gpurun_out/r03m/mfma.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03m/trace -o run --output-format csv -- python3 $R/bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline --no-overlap > $R/gpurun_out/r03m/trace.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/r03m/mfma gram_dense > $R/gpurun_out/r03m/mfma_summary.json && cat $R/gpurun_out/r03m/mfma_summary.json && grep gram_dense $R/gpurun_out/r03m/trace/run_kernel_stats.csv
