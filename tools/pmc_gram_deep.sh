#!/bin/bash
# latency / occupancy counters of the Gram kernel alone (tools/gram_one.py), one pass per group
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-pmc_deep}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAVES" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES" \
           "SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_VMEM_TA_ADDR_FIFO_FULL" \
           "SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $O/g$i -o run --output-format csv -- python3 $R/tools/gram_one.py 100000 4096 > $O/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/g$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O gram_sparse > $O/summary.json && cat $O/summary.json
