#!/bin/bash
# double-buffered dense MFMA Gram (GRF_DENSE_DB) A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread -k "dense or gpflow" > gpurun_out/dense7.log 2>&1 || { tail -30 gpurun_out/dense7.log; exit 1; }
tail -1 gpurun_out/dense7.log
for db in 0 1 0 1; do GRF_DENSE_DB=$db timeout -k 10 120 python tools/dense_sweep.py 2708 4096 10000 16384 | sed "s/^/DB=$db /" || exit 1; done
