set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "walk_phi or phi or heavy or sharded or snap or full_pipeline or smoke or cora or steps" > gpurun_out/gpu_walk.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python3 tools/walkphi_ab.py c4 && timeout -k 10 300 python3 tools/walkphi_ab.py c5 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK && \
timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && echo C5_OK
