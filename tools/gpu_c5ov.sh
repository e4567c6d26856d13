set -o pipefail
mkdir -p gpurun_out
for ov in --no-overlap --overlap --no-overlap --overlap; do
timeout -k 10 400 python bench.py --workload c5 --steps 4 --warmup 1 --no-cpu-baseline $ov > gpurun_out/c5ov.json 2> gpurun_out/c5ov.err && echo "$ov $(python -c "import json;d=json.load(open('gpurun_out/c5ov.json'));print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), d['serial_ms_per_step'])")" || exit 1
done
