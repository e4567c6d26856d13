#!/bin/bash
# C5 column-block Gram: band width of the own-rows transpose (8192 = one band of 8-wave tiles, 2 per CU;
# 4096 / 2048 = two / four bands of 4-wave tiles, 4 / 6 per CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/c5bw
mkdir -p $O
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-mfma-leg --workload c5 --steps 5 --warmup 2 "$@" > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$* $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
run --band-width 8192
run --band-width 4096
run --band-width 2048
run --band-width 6144
run --band-width 8192
run --band-width 4096
