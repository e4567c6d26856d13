#!/bin/bash
# list tiles for sparse buckets (column-block Gram): parity, then the C5 bench
set -o pipefail
mkdir -p gpurun_out/list
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "column_block or sharded or degenerate" > gpurun_out/list/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/list/c5.json 2> gpurun_out/list/c5.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/list/c5.json').read().strip().splitlines()[-1]);print('c5', round(d['ms_per_step'],2), 'gram', round(d['roofline']['kernel_ms'],2))"
done
