#!/bin/bash
# fused symmetric completion: bit-equality tests, then a same-box A/B against tiles + mirror
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fused
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "gram_sparse_vs_oracle or degenerate" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 "$@" > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$* $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
run --no-fused
run --fused
run --fused --front-at 0.9
run --fused --front-at 0.8
run --fused --front-at 0.6
run --no-fused
run --fused
