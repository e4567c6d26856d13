set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench10.json 2> gpurun_out/bench10.err && echo BENCH10_OK
