#!/bin/bash
# Philox rounds with 64-bit products: walk parity, then walk_phi / step timing (compare with the previous commit's numbers)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/philox64
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_estimator.py -x -q --timeout 200 --timeout-method thread \
    -k "philox or walk or bench_path or estimator or clt or augmented" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg "$@" > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$* $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline_walk']['kernel_ms'],3), round(d['serial_ms_per_step'],2))")"
}
run --steps 10
run --workload c5 --steps 5
run --steps 10
run --workload c5 --steps 5
