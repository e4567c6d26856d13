#!/bin/bash
# Round 4: walk divide/normalise changes -- bit-exactness subset, C4 / C5 benches, walk VALU PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_run4
mkdir -p $O
cd $R
bash tools/gpu_tests.sh r04_run4_tests "walk or phi or headline or degenerate or estimator or steps or snap or golden or api or features" 900 || exit 1
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
echo bench ok; tail -c 300 $O/bench.json
timeout -k 10 400 python3 -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail $O/bench_c5.err; exit 1; }
echo c5 ok; tail -c 300 $O/bench_c5.json
PASSES=sq timeout -k 10 500 $R/tools/pmc_passes.sh $O/pmc_c4 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-mfma-leg || exit 1
echo done
