#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, --pmc only: no trace domains) over a command.
# usage: tools/pmc_passes.sh <outdir> <python args...>   (runs: python3 <args> under each pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# PASSES="fetch write ..." runs only those passes (default: all five)
PASSES=${PASSES:-fetch write sq lds ta}
run() {
    local name=$1; shift
    case " $PASSES " in *" $name "*) ;; *) return 0;; esac
    timeout -k 10 420 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "${ARGS[@]}" \
        > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -20 "$OUT/$name.log"; exit 1; }
    echo "pass $name ok"
}
ARGS=("$@")
run fetch FETCH_SIZE
run write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
# (GRBM_GUI_ACTIVE in the same pass as SQ_INSTS_VALU: the walk's VALU rate comes from one pass)
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
run lds SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
run ta TA_BUSY_avr TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
