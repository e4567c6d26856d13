#!/bin/bash
# self-counting transpose: parity tests, then bench A/B against the walk-counted plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "Error|assert" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for s in 1 0 1 0; do
  GRF_TRANSPOSE_SELF=$s timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "self=$s $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2), round(d['roofline_walk']['kernel_ms'],3))")"
done
for s in 1 0; do
  GRF_TRANSPOSE_SELF=$s timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline --steps 10 > $O/c5.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "c5 self=$s $(python -c "import json;d=json.loads(open('$O/c5.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['serial_ms_per_step'],2), round(d['roofline_walk']['kernel_ms'],3))")"
done
