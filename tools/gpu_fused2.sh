#!/bin/bash
# fused completion decomposition (GRF_FUSE_EXP timing-only variants: 1 nt row stores, 2 no completion, 4 no acquire)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fused2
mkdir -p $O
run() {
  GRF_FUSE_EXP=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 10 --warmup 2 --fused --no-overlap > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "exp=$1 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))")"
}
for e in 24 88 152 216; do run $e; done
