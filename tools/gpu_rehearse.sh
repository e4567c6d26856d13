# multi-process rehearsal of bench.py's N > 1 path on ONE GPU (gloo, host-staged collectives)
set -o pipefail
mkdir -p gpurun_out
export GRF_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/reh2.json 2> gpurun_out/reh2.err && echo REH2_OK && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/reh3.json 2> gpurun_out/reh3.err && echo REH3_OK && \
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --n-nodes 20000 --edges 200000 --mode allreduce > gpurun_out/reh2ar.json 2> gpurun_out/reh2ar.err && echo REH2AR_OK
