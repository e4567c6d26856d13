#!/bin/bash
# split-K dense Gram with the slice as the fastest workgroup index (one XCD per slice at 8 slices)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "dense" > gpurun_out/dense6.log 2>&1 || { tail -30 gpurun_out/dense6.log; exit 1; }
tail -1 gpurun_out/dense6.log
for sp in 0 2 4 8; do GRF_DENSE_SPLIT=$sp timeout -k 10 120 python tools/dense_sweep.py 2708 4096 6000 8192 10000 | sed "s/^/S=$sp /" || exit 1; done
