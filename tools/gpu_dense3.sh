#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "gram_dense" > gpurun_out/dense3.log 2>&1 || { tail -30 gpurun_out/dense3.log; exit 1; }
tail -1 gpurun_out/dense3.log
timeout -k 10 120 python tools/dense_sweep.py 2708 4096 10000 || exit 1
GRF_DENSE_SPLIT=1 timeout -k 10 120 python tools/dense_sweep.py 2708 || exit 1
GRF_DENSE_SPLIT=2 timeout -k 10 120 python tools/dense_sweep.py 2708 || exit 1
GRF_DENSE_SPLIT=3 timeout -k 10 120 python tools/dense_sweep.py 2708 || exit 1
GRF_DENSE_SPLIT=4 timeout -k 10 120 python tools/dense_sweep.py 2708 4096 || exit 1
GRF_DENSE_SPLIT=8 timeout -k 10 120 python tools/dense_sweep.py 2708 4096 || exit 1
timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --steps 20 > gpurun_out/dense3_c3.json 2>&1 && tail -1 gpurun_out/dense3_c3.json
timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 10 > gpurun_out/dense3_c2.json 2>&1 && tail -1 gpurun_out/dense3_c2.json
