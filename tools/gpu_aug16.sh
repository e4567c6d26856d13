#!/bin/bash
# 16-byte augmented walk records: parity, then C5 / C4 A/B against the 32-byte records (GRF_WALK_AUG16=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/aug16
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread \
    -k "augmented or walk_phi or bench_path or philox or degenerate or snap" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg ${@:2} > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$1 ${@:2} $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline_walk']['kernel_ms'],3), round(d['serial_ms_per_step'],2))")"
}
run GRF_WALK_AUG16=0 --workload c5 --steps 5
run GRF_WALK_AUG16=1 --workload c5 --steps 5
run GRF_WALK_AUG16=0 --steps 10
run GRF_WALK_AUG16=1 --steps 10
run GRF_WALK_AUG16=0 --workload c5 --steps 5
run GRF_WALK_AUG16=1 --workload c5 --steps 5
