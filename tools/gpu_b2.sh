set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "api or gpflow or gptorch or phi or snap" > gpurun_out/gpu_b2.log 2>&1 && echo TESTS_OK && \
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_b$i.json 2> gpurun_out/bench_b.err && echo "B$i $(python -c "import json;d=json.load(open('gpurun_out/bench_b$i.json'));print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")" || exit 1; done
