set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "transpose or heavy or sharded or walk_phi" > gpurun_out/gpu_tr.log 2>&1 && echo TESTS_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK && \
bash tools/trace_c5.sh
