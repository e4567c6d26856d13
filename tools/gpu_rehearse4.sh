#!/bin/bash
# N = 4 bench path rehearsed with gloo ranks on one GPU (C4 column blocks with the symmetric square, exact Phi gather)
set -o pipefail
mkdir -p gpurun_out/reh4
export GRF_DIST_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 \
    bench.py --gpus 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/reh4/c4.json 2> gpurun_out/reh4/c4.err && echo C4_N4_OK && \
    cut -c1-300 gpurun_out/reh4/c4.json
