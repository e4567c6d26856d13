#!/bin/bash
# Gram windows in flight per wave: 8 (default) vs 12 (114 VGPRs, still 4 waves per SIMD), interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/unroll12
mkdir -p $O
run() {
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$1 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
for i in 1 2; do run GRF_GRAM_UNROLL=8; run GRF_GRAM_UNROLL=12; run GRF_GRAM_UNROLL=16; done
