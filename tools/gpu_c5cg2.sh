set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "cg or spmm or predict or matvec or csr_transpose" > gpurun_out/gpu_cg.log 2>&1 && echo CGTESTS_OK && \
timeout -k 10 500 python bench.py --workload predict --graph powerlaw --n 1000000 --walks 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5pred.json 2> gpurun_out/bench_c5pred.err && echo C5PRED_OK && \
timeout -k 10 300 python bench.py --workload predict --steps 5 --warmup 1 > gpurun_out/bench_pred.json 2> gpurun_out/bench_pred.err && echo PRED_OK
