#!/bin/bash
# eight-rows-per-wave sparse Laplacian: parity, then C5 kernel stats against one row per wave
set -o pipefail
mkdir -p gpurun_out/lap
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_api.py \
    -k "laplacian or snap or heavy or degenerate or cora or entry_points or samplers or pcg64" > gpurun_out/lap/tests.log 2>&1 || exit 1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  GRF_LAP_WAVE_ROWS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/lap/t$v -o run --output-format csv -- \
      python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/lap/c5_$v.json 2> $R/gpurun_out/lap/c5_$v.err || exit 1
done
cd $R
for v in 0 1; do python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/lap/t$v/run_kernel_stats.csv')))
print('wave_rows=$v', [(x['Name'][:24], round(float(x['AverageNs'])/1e3,1)) for x in rows if 'lap' in x['Name']])
"; done
