#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/gpu_tests.sh r04_run5_tests "transpose or gram or snap or hub or heavy or powerlaw or degenerate or cols or sharded" 900 || exit 1
bash tools/r04_trace_social.sh || exit 1
for g in enron facebook; do
  timeout -k 10 300 python3 -u bench.py --graph $g --no-cpu-baseline > gpurun_out/r04_social/bench_$g.json 2> gpurun_out/r04_social/bench_$g.err || { echo "$g bench failed"; exit 1; }
  tail -c 250 gpurun_out/r04_social/bench_$g.json; echo
done
