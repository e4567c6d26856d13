set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 300 python3 tools/overlap_events.py 1024 > gpurun_out/r03c/overlap.json 2> gpurun_out/r03c/overlap.err && cat gpurun_out/r03c/overlap.json && \
timeout -k 10 300 python3 tools/gram_crossover.py > gpurun_out/r03c/crossover.txt 2> gpurun_out/r03c/crossover.err && cat gpurun_out/r03c/crossover.txt && \
timeout -k 10 300 python3 bench.py --workload c2 --path sparse > gpurun_out/r03c/bench_c2_sparse.json 2> gpurun_out/r03c/bench_c2_sparse.err && tail -c 400 gpurun_out/r03c/bench_c2_sparse.json && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-mfma-leg > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err && python3 -c "import json;d=json.loads(open('gpurun_out/r03c/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['serial_ms_per_step'],d['roofline']['kernel_ms'])"
