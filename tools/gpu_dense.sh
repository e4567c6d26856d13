set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or cora or entry_points or gpflow" > gpurun_out/gpu_dense.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && echo C3_OK
bash tools/pmc_dense.sh
