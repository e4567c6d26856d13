#!/bin/bash
# round-2 refresh of the tree after the walk_phi scan/sort changes: full GPU suite, smoke, headline bench + traces + PMC, C5 trace,
# gloo rehearsal of the N > 1 bench paths
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r02s
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo gpu tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
$R/tools/gpu_profile.sh r02s/prof || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- \
    python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/trace_c5.log 2>&1 || { echo trace c5 failed; tail $O/trace_c5.log; exit 1; }
echo trace c5 ok
cd $R
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 bench failed; tail $O/bench_c5.err; exit 1; }
echo c5 bench ok
bash tools/gpu_rehearse3.sh || { echo rehearsal failed; exit 1; }
