#!/bin/bash
# C5 column block against the block transpose's band width
set -o pipefail
mkdir -p gpurun_out/c5cb
for bw in 8192 4096 2048 8192; do
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline --band-width $bw > gpurun_out/c5cb/b.json 2> gpurun_out/c5cb/b.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/c5cb/b.json').read().strip().splitlines()[-1]);print('bw=$bw', round(d['ms_per_step'],2), 'gram', round(d['roofline']['kernel_ms'],2))"
done
