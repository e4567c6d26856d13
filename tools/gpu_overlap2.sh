set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s$i.json 2> gpurun_out/bench_s$i.err && echo SERIAL_OK && \
timeout -k 10 300 python bench.py --no-cpu-baseline --overlap --steps 10 > gpurun_out/bench_o$i.json 2> gpurun_out/bench_o$i.err && echo OV_OK || exit 1
done
