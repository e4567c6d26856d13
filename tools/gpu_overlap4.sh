set -o pipefail
mkdir -p gpurun_out
for fa in 1.0 0.9 0.8 1.0 0.9 0.8; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --front-at $fa > gpurun_out/bench_fa$fa.json 2> gpurun_out/bench_fa.err && echo "fa=$fa $(python -c "import json;d=json.load(open('gpurun_out/bench_fa$fa.json'));print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")" || exit 1
done
