set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ov.json 2> gpurun_out/bench_ov.err && echo OV_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-overlap > gpurun_out/bench_noov.json 2> gpurun_out/bench_noov.err && echo NOOV_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_ov10.json 2> gpurun_out/bench_ov10.err && echo OV10_OK
