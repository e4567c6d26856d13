#!/bin/bash
# N > 1 bench paths rehearsed with gloo ranks on one GPU: C4 column blocks (2 ranks), C5 column blocks (2 ranks)
set -o pipefail
mkdir -p gpurun_out/reh3
export GRF_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/reh3/c4.json 2> gpurun_out/reh3/c4.err && echo C4_OK && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --workload c5 > gpurun_out/reh3/c5.json 2> gpurun_out/reh3/c5.err && echo C5_OK
