#!/bin/bash
# int32 wave scans in DPP steps everywhere (walk, transpose, steps): parity, then prev/new library A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/dppscan2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env GRF_AMD_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg $3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$2 $3 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline_walk']['kernel_ms'],3), round(d['serial_ms_per_step'],2))")"
}
P=tools/libgrf_prev.so; N=efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so
for i in 1 2; do run $P prev "--steps 20"; run $N new "--steps 20"; done
for i in 1 2; do run $P prev "--workload c5 --steps 5"; run $N new "--workload c5 --steps 5"; done
