set -o pipefail
mkdir -p gpurun_out
for w in 0 512 768 1024 0 512 768 1024; do
GRF_MIRROR_WGS=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench_mw$w.json 2> gpurun_out/bench_mw.err && echo "wgs=$w $(python -c "import json;d=json.load(open('gpurun_out/bench_mw$w.json'));print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")" || exit 1
done
