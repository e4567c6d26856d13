#!/bin/bash
# C5 Gram (8192-row block, packed records) against the tile knobs: unroll, waves per tile, exact tail
set -o pipefail
mkdir -p gpurun_out/c5g
: > gpurun_out/c5g/log
for cfg in "8 0 1" "4 0 1" "16 0 1" "8 4 1" "8 0 0"; do
  set -- $cfg
  GRF_GRAM_UNROLL=$1 GRF_GRAM_WAVES=$2 GRF_GRAM_TAIL=$3 timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --steps 5 > gpurun_out/c5g/b.json 2> gpurun_out/c5g/b.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/c5g/b.json').read().strip().splitlines()[-1]);print('unroll=$1 waves=$2 tail=$3', round(d['ms_per_step'],2), 'gram', round(d['roofline']['kernel_ms'],2))" >> gpurun_out/c5g/log
done
cat gpurun_out/c5g/log
