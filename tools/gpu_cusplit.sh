#!/bin/bash
# pipelined C4 step with the next front and the mirror on disjoint CUs (CU-masked streams)
set -o pipefail
mkdir -p gpurun_out/cus
: > gpurun_out/cus/log
for cfg in "0 0" "0.5 0" "0.25 0" "0.5 1024" "0.333 0" "0 0"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --cu-split $1 --mirror-wgs $2 > gpurun_out/cus/b.json 2> gpurun_out/cus/b.err || { tail -5 gpurun_out/cus/b.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/cus/b.json').read().strip().splitlines()[-1]);print('split=$1 wgs=$2', round(d['ms_per_step'],2), 'serial', round(d['serial_ms_per_step'],2))" >> gpurun_out/cus/log
done
cat gpurun_out/cus/log
