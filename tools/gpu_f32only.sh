#!/bin/bash
# walk_phi without the float64 Phi copy on the bench paths: parity, then C4 / C5 benches
set -o pipefail
mkdir -p gpurun_out/f32
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "walk_phi or degenerate or heavy or sharded or column_block or c2_scale" > gpurun_out/f32/tests.log 2>&1 || exit 1
for w in kernel c5 kernel c5; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/f32/b.json 2> gpurun_out/f32/b.err || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/f32/b.json').read().strip().splitlines()[-1]);print('$w', round(d['ms_per_step'],2))"
done
