set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmcdense
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES -d $O/p1 -o run --output-format csv -- python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/p1.log 2>&1 && echo PMC_OK
python3 $R/tools/pmc_summary.py $O gram_dense > $O/summary.json && echo SUM_OK
