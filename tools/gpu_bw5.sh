#!/bin/bash
# band widths whose tile fits 5 per CU (W*8 + 8 KB <= 32 KB) against the 4096 default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/bw5
mkdir -p $O
run() {
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 10 --warmup 2 "$@" > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$* $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
run --band-width 4096
run --band-width 3072
run --band-width 2560
run --band-width 3584
run --band-width 4096
run --band-width 3072
