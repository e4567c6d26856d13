set -o pipefail
mkdir -p gpurun_out
for tb in 0 67108864 268435456; do
GRF_SPMM_TILE_BYTES=$tb timeout -k 10 300 python bench.py --workload predict --graph powerlaw --n 1000000 --walks 64 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5cg_$tb.json 2> gpurun_out/c5cg.err && echo "tb=$tb $(python -c "import json;d=json.load(open('gpurun_out/c5cg_$tb.json'));print(round(d['ms_per_step'],1), d['config']['cg_iterations'], round(d['roofline']['kernel_ms'],2))")" || exit 1
done
