set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_o$i.json 2> gpurun_out/bench_o$i.err && echo OV_OK || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_o20.json 2> gpurun_out/bench_o20.err && echo OV20_OK
