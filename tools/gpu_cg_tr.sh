#!/bin/bash
# CSR transpose by radix sort: CG parity tests, then the C4 predict workload
set -o pipefail
mkdir -p gpurun_out/cgtr
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_cg.py > gpurun_out/cgtr/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload predict --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/cgtr/pred.json 2> gpurun_out/cgtr/pred.err || exit 1
python3 -c "
import json;d=json.loads(open('gpurun_out/cgtr/pred.json').read().strip().splitlines()[-1]);print('predict', round(d['ms_per_step'],2))"
