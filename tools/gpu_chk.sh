set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err && echo BENCH_OK && \
bash tools/trace_c5.sh
