#!/bin/bash
# C5 K block as a column block from the block rows' transpose vs the row block from the full transpose
set -o pipefail
mkdir -p gpurun_out/c5c
for mode in cols rows cols; do
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --mode $mode > gpurun_out/c5c/$mode.json 2> gpurun_out/c5c/$mode.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/c5c/$mode.json').read().strip().splitlines()[-1]);print('$mode', round(d['ms_per_step'],2), round(d['value']), 'gram', round(d['roofline']['kernel_ms'],2))"
done
