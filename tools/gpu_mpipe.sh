#!/bin/bash
# mirror with the next block's loads in flight (GRF_MIRROR_PIPE): parity, then a same-box A/B and grid sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/mpipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "gram_sparse_vs_oracle or degenerate or dense" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$1 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
run GRF_MIRROR_PIPE=0
run GRF_MIRROR_PIPE=1
run GRF_MIRROR_WGS=768
run GRF_MIRROR_WGS=1536
run GRF_MIRROR_WGS=2048
run GRF_MIRROR_WGS=512
run GRF_MIRROR_PIPE=0
run GRF_MIRROR_PIPE=1
