#!/bin/bash
# column-block multi-GPU Gram: parity, per-rank compute emulated on one GPU, 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "column_block or sharded or gram_sparse_vs_oracle" > gpurun_out/cols_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/cols_emul.py 2,4,8 3 > gpurun_out/cols_emul.json 2>&1 && \
GRF_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/reh2cols.json 2> gpurun_out/reh2cols.err && echo REH2COLS_OK
rc=$?; tail -3 gpurun_out/cols_tests.log; cat gpurun_out/cols_emul.json; tail -c 400 gpurun_out/reh2cols.json; exit $rc
