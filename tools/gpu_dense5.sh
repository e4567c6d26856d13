#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread -k "dense or gpflow or c3" > gpurun_out/dense5.log 2>&1 || { tail -30 gpurun_out/dense5.log; exit 1; }
tail -1 gpurun_out/dense5.log
timeout -k 10 120 python tools/dense_sweep.py 2708 4096 6000 8192 10000 || exit 1
timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --steps 20 > gpurun_out/dense5_c3.json 2>&1 && tail -1 gpurun_out/dense5_c3.json
timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 10 > gpurun_out/dense5_c2.json 2>&1 && tail -1 gpurun_out/dense5_c2.json
