#!/bin/bash
# Gram tile nonzero order (GRF_GRAM_ORDER 0 contiguous / 1 interleaved / 2 interleaved + shared phase):
# parity under each order, then a same-box interleaved A/B of the C4 pipelined bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/order
mkdir -p $O
for o in 1 2; do
  GRF_GRAM_ORDER=$o timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "gram or degenerate or bench_path or column_block" > $O/tests$o.log 2>&1 || { echo tests $o failed; tail -30 $O/tests$o.log; exit 1; }
  echo "order $o: $(tail -1 $O/tests$o.log)"
done
run() {
  env GRF_GRAM_ORDER=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "order $1 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
for i in 1 2; do run 0; run 1; run 2; done
