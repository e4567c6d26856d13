#!/bin/bash
# striped (LDS-transposed) scans vs the per-lane-run kernels: parity tests, then C5 kernel stats of both
set -o pipefail
mkdir -p gpurun_out/scan
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "transpose or laplacian or steps_and_phi or sharded or gram_sparse_vs_oracle or degenerate" > gpurun_out/scan/tests.log 2>&1 || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  GRF_SCAN_LEGACY=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/scan/t$v -o run --output-format csv -- \
      python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/scan/c5_$v.json 2> $R/gpurun_out/scan/c5_$v.err || exit 1
done
cd $R
for v in 0 1; do python3 -c "
import csv,json
d=json.loads(open('gpurun_out/scan/c5_$v.json').read().strip().splitlines()[-1])
rows=list(csv.DictReader(open('gpurun_out/scan/t$v/run_kernel_stats.csv')))
print('legacy=$v', round(d['ms_per_step'],2), [(x['Name'][:28], x['Calls'], round(float(x['AverageNs'])/1e6,3)) for x in rows if 'scan' in x['Name']])
"; done
