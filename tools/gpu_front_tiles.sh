#!/bin/bash
# the next front beside the Gram tiles (front-at 0) with fewer tiles per CU (GRF_GRAM_LDS_PAD) vs beside the mirror
set -o pipefail
mkdir -p gpurun_out/ft
: > gpurun_out/ft/log
for cfg in "1.0 0" "0.0 0" "0.0 8192" "1.0 8192" "0.0 4096"; do
  set -- $cfg
  GRF_GRAM_LDS_PAD=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --front-at $1 > gpurun_out/ft/b.json 2> gpurun_out/ft/b.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/ft/b.json').read().strip().splitlines()[-1]);print('front_at=$1 pad=$2', round(d['ms_per_step'],2), 'serial', round(d['serial_ms_per_step'],2), 'K', round(d['roofline']['kernel_ms'],2))" >> gpurun_out/ft/log
done
cat gpurun_out/ft/log
