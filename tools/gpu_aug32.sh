#!/bin/bash
# 32-byte augmented walk records: parity, then walk_phi at C5 / C4 (aug vs plain CSR walk) and the C5 bench
set -o pipefail
mkdir -p gpurun_out/aug
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "walk_phi or degenerate or heavy or c3 or dense or column_block" > gpurun_out/aug/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/walkphi_ab.py c5 count,noaug,count > gpurun_out/aug/c5.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/walkphi_ab.py c4 count,noaug,count > gpurun_out/aug/c4.json 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > gpurun_out/aug/b5.json 2> gpurun_out/aug/b5.err || exit 1
tail -n1 gpurun_out/aug/c5.json gpurun_out/aug/c4.json
python3 -c "
import json;d=json.loads(open('gpurun_out/aug/b5.json').read().strip().splitlines()[-1]);print('c5 bench', round(d['ms_per_step'],2))"
