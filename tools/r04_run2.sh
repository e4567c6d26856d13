#!/bin/bash
# Round 4: VALU ceiling (mad_u64, med3 added), C5 band-width A/B, dense MFMA busy PMC (default IL=2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_run2
mkdir -p $O
cd $R
bash tools/gpu_tests.sh r04_run2_tests "gram_dense" 300 || exit 1
timeout -k 10 120 ./tools/valu_ceiling > $O/valu_ceiling.txt 2>&1 || { echo valu failed; exit 1; }
cat $O/valu_ceiling.txt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d $O/dense_pmc -o run --output-format csv -- python3 $R/tools/dense_ab.py --reps 3 10000 2708 > $O/dense_pmc.log 2>&1) || { echo dense pmc failed; tail $O/dense_pmc.log; exit 1; }
echo dense pmc ok
bash tools/gpu_ab.sh r04_c5_band "bench.py --workload c5 --no-cpu-baseline --steps 10 --warmup 2" "X=0" "X=0 :: --band-width 4096" || exit 1
cat gpurun_out/r04_c5_band/ab.txt | cut -c1-300
