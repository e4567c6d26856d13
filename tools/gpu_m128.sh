#!/bin/bash
# 128 x 128-block mirror (GRF_MIRROR_128=1): parity with it on, then an interleaved A/B (pipelined and serial)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/m128
mkdir -p $O
GRF_MIRROR_128=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread \
    -k "gram or degenerate or dense or bench_path or entry_points" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 $2 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$1 $2 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
for i in 1 2 3; do run GRF_MIRROR_128=0; run GRF_MIRROR_128=1; done
run GRF_MIRROR_128=0 --no-overlap
run GRF_MIRROR_128=1 --no-overlap
