#!/bin/bash
# scans / fused transpose plan: parity tests, then the C5 kernel stats
set -o pipefail
mkdir -p gpurun_out/scan
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "transpose or laplacian or steps_and_phi or sharded or gram_sparse_vs_oracle or degenerate or column_block" > gpurun_out/scan/tests.log 2>&1 || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/scan/t -o run --output-format csv -- \
    python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/scan/c5.json 2> $R/gpurun_out/scan/c5.err || exit 1
cd $R
python3 -c "
import csv,json
d=json.loads(open('gpurun_out/scan/c5.json').read().strip().splitlines()[-1])
rows=list(csv.DictReader(open('gpurun_out/scan/t/run_kernel_stats.csv')))
print(round(d['ms_per_step'],2), [(x['Name'][:28], x['Calls'], round(float(x['AverageNs'])/1e6,3)) for x in rows][:14])
"
