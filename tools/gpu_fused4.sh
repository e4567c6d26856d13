#!/bin/bash
# fused completion: store flavour of the transposed block (GRF_FUSE_EXP 64 plain, 128 sc1, 0 nt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fused4
mkdir -p $O
run() {
  GRF_FUSE_EXP=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 10 --warmup 2 "${@:2}" > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "exp=$1 ${@:2} $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
run 64 --fused --no-overlap
run 128 --fused --no-overlap
run 0 --fused --no-overlap
