#!/bin/bash
# Bench + kernel-trace stats + PMC passes for the headline config (writes gpurun_out/<tag>/).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-prof}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
echo bench ok; cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mfma-leg > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
echo trace ok
# the MFMA leg's kernels (C3 dense path) in a trace of their own (per-kernel averages stay per workload)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c3 -o run --output-format csv -- \
    python3 $R/bench.py --workload c3 --steps 20 --warmup 2 --no-cpu-baseline > $O/trace_c3.log 2>&1 || { echo trace c3 failed; tail $O/trace_c3.log; exit 1; }
echo trace c3 ok
$R/tools/pmc_passes.sh $O/pmc $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-mfma-leg || exit 1
python3 $R/tools/pmc_summary.py $O/pmc > $O/pmc_summary.json && echo pmc ok
