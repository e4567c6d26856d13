#!/bin/bash
# The dense-path records: the headline line (its MFMA legs), the C2 / C3 lines, their kernel traces and one PMC
# pass (MFMA busy) of the C2 Gram.  usage: tools/gpu_dense_final.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-dense_final}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_headline.py -m gpu -k "gram_dense or c3_dense_leg" > $O/tests.log 2>&1 || { echo tests failed; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload c2 > $O/c2.json 2> $O/c2.err || { echo c2 failed; exit 1; }
timeout -k 10 300 python3 bench.py --workload c3 > $O/c3.json 2> $O/c3.err || { echo c3 failed; exit 1; }
echo lines ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o run --output-format csv -- \
    python3 $R/bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline > $O/trace_c3.log 2>&1 || { echo trace c3 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- \
    python3 $R/bench.py --workload c2 --steps 10 --warmup 2 --no-cpu-baseline > $O/trace_c2.log 2>&1 || { echo trace c2 failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc1 -o run --output-format csv -- python3 $R/tools/dense_ab.py --reps 3 2708 10000 \
    > $O/pmc1.log 2>&1 || { echo pmc failed; exit 1; }
echo traces ok
