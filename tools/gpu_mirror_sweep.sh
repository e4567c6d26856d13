#!/bin/bash
# pipelined C4 step against the mirror's grid (GRF_MIRROR_WGS), same box
set -o pipefail
mkdir -p gpurun_out/ms
: > gpurun_out/ms/log
for w in 1024 768 1536 2048 1024 512; do
  GRF_MIRROR_WGS=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ms/b.json 2> gpurun_out/ms/b.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/ms/b.json').read().strip().splitlines()[-1]);print('wgs=$w', round(d['ms_per_step'],2), 'serial', round(d['serial_ms_per_step'],2))" >> gpurun_out/ms/log
done
cat gpurun_out/ms/log
