#!/bin/bash
# walk_phi: one slot carries the source's step-0 run: parity, then prev / new library A/B (C4, C5)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/step0
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_estimator.py -x -q --timeout 120 --timeout-method thread \
    -k "walk or phi or bench_path or estimator or degenerate" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env GRF_AMD_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 10 --warmup 2 $3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$2 $3 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['serial_ms_per_step'],2), round(d.get('roofline_walk',{}).get('kernel_ms',0),3))")"
}
for i in 1 2; do
  run tools/libgrf_prev.so prev ""; run efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so new ""
  run tools/libgrf_prev.so prev "--workload c5"; run efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so new "--workload c5"
done
