#!/bin/bash
# refresh the secondary workload bench lines with the current code (each with its CPU baseline)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/wl_r02
mkdir -p $O
timeout -k 10 300 python bench.py --graph enron > $O/enron.json 2> $O/enron.err || { tail $O/enron.err; exit 1; }
echo enron ok
timeout -k 10 300 python bench.py --graph facebook > $O/facebook.json 2> $O/facebook.err || { tail $O/facebook.err; exit 1; }
echo facebook ok
timeout -k 10 400 python bench.py --workload c5 > $O/c5.json 2> $O/c5.err || { tail $O/c5.err; exit 1; }
echo c5 ok
timeout -k 10 300 python bench.py --workload predict > $O/predict.json 2> $O/predict.err || { tail $O/predict.err; exit 1; }
echo predict ok
timeout -k 10 300 python bench.py --no-sym --no-cpu-baseline > $O/rows.json 2> $O/rows.err || { tail $O/rows.err; exit 1; }
echo rows ok
timeout -k 10 300 python bench.py --workload c3 > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
echo c3 ok
