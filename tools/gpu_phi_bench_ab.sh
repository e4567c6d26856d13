set -o pipefail
mkdir -p gpurun_out
for t in 256 128 256 128; do
GRF_PHI_THREADS=$t timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_t$t.json 2> gpurun_out/bench_t.err && echo "T=$t $(python -c "import json;d=json.load(open('gpurun_out/bench_t$t.json'));print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")" || exit 1
done
