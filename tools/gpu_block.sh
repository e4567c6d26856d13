#!/bin/bash
# block-symmetric row blocks: parity + per-rank timing (row mode vs block-symmetric) at N = 2, 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "block_symmetric or gram_sparse_vs_oracle" > gpurun_out/block_tests.log 2>&1 && \
GRF_BW=8192 timeout -k 10 240 python -u tools/gram_time.py 100000 3 blocks2,blocks4 > gpurun_out/block_time.json 2>&1
rc=$?; tail -3 gpurun_out/block_tests.log; cat gpurun_out/block_time.json; exit $rc
