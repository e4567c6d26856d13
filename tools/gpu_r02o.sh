#!/bin/bash
# final round-2 profile of the current tree: smoke, headline bench + kernel-trace stats (C4, C3) + PMC, C5 trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r02o
mkdir -p $O
cd $R
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$R/tools/gpu_profile.sh r02o/prof || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- \
    python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/trace_c5.log 2>&1 || { echo trace c5 failed; tail $O/trace_c5.log; exit 1; }
echo trace c5 ok
