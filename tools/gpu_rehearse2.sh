set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sym > gpurun_out/rows_serial.json 2> gpurun_out/rows.err && echo RS_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sym --overlap > gpurun_out/rows_ov.json 2> gpurun_out/rows.err && echo RO_OK && \
GRF_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --overlap > gpurun_out/reh2ov.json 2> gpurun_out/reh2ov.err && echo REH2OV_OK
