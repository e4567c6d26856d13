#!/bin/bash
# Every secondary bench workload once (one JSON line each under gpurun_out/wl/), plus the C5 kernel stats.
set -o pipefail
O=gpurun_out/wl
mkdir -p $O
run() {  # run <name> <timeout> <bench args...>
    local name=$1 t=$2; shift 2
    timeout -k 10 $t python -u bench.py "$@" > $O/$name.json 2> $O/$name.err && echo "$name ok $(tail -c 300 $O/$name.json)"
}
run enron 300 --graph enron && \
run facebook 300 --graph facebook && \
run c5 400 --workload c5 && \
run c2 300 --workload c2 && \
run c2_sparse 300 --workload c2 --path sparse && \
run rows 300 --no-sym && \
run predict 300 --workload predict --steps 5 --warmup 1 && \
run c3 300 --workload c3 && \
run c5_predict 500 --workload predict --graph powerlaw --n 1000000 --walks 64 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/c5trace -o run --output-format csv -- \
    python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/c5trace.log 2>&1 && echo c5 trace ok
