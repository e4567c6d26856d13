set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "snap or heavy_tailed" > gpurun_out/gpu_snap.log 2>&1 && echo SNAP_TESTS_OK && \
timeout -k 10 300 python bench.py --graph enron --steps 5 --warmup 2 > gpurun_out/bench_enron.json 2> gpurun_out/bench_enron.err && echo ENRON_OK && \
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && echo C5_OK
