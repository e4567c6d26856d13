set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "laplacian or snap or heavy_tailed or c2_scale or entry_points or samplers" > gpurun_out/gpu_lap.log 2>&1 && echo LAP_TESTS_OK && \
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && echo C5_OK
