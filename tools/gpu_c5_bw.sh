#!/bin/bash
# C5 step at several transpose band widths (row-mode Gram of an 8192-row block)
set -o pipefail
mkdir -p gpurun_out/c5bw
: > gpurun_out/c5bw/log
for bw in 8192 4096 2048 8192; do
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --band-width $bw > gpurun_out/c5bw/c5.json 2> gpurun_out/c5bw/c5.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/c5bw/c5.json').read().strip().splitlines()[-1]);print('bw=$bw', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))" >> gpurun_out/c5bw/log
done
cat gpurun_out/c5bw/log
