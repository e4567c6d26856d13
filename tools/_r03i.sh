set -o pipefail
mkdir -p gpurun_out/r03i
bash tools/gpu_tests.sh r03i "" 1000 && \
timeout -k 10 600 python3 tools/balance_emul.py enron,facebook,powerlaw200k 4,8 3 > gpurun_out/r03i/balance.jsonl 2> gpurun_out/r03i/balance.err && cat gpurun_out/r03i/balance.jsonl
