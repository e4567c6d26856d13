#!/bin/bash
# Gram exact tail groups masking only their last window: parity, then a same-box A/B against the previous build
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dppscan
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "gram or degenerate or bench_path or sharded_counts or column_block" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env GRF_AMD_LIB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$3 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
for i in 1 2 3; do run x tools/libgrf_prev.so prev; run x efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so new; done
