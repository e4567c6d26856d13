set -o pipefail
mkdir -p gpurun_out
for cfg in "GRF_BENCH_PRIO=0" "GRF_BENCH_PRIO=1" "GRF_BENCH_PRIO=1 GRF_MIRROR_WGS=0" "GRF_BENCH_PRIO=1 GRF_MIRROR_WGS=2048" "GRF_BENCH_PRIO=0" "GRF_BENCH_PRIO=1"; do
env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err && echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/bench_p.json'));print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")" || exit 1
done
