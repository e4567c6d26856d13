#!/bin/bash
# C5 bench line (with the CPU baseline) + kernel stats
set -o pipefail
mkdir -p gpurun_out/c5p
timeout -k 10 400 python -u bench.py --workload c5 > gpurun_out/c5p/c5.json 2> gpurun_out/c5p/c5.err || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c5p/trace -o run --output-format csv -- \
    python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/c5p/trace.log 2>&1 && echo c5 trace ok
