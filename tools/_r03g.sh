set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 120 tools/lds_bench > gpurun_out/r03g/lds_bench.txt 2>&1 && cat gpurun_out/r03g/lds_bench.txt && \
timeout -k 10 300 python3 tools/kblock_density.py > gpurun_out/r03g/kblock_density.json 2> gpurun_out/r03g/kblock_density.err && cat gpurun_out/r03g/kblock_density.json && \
bash tools/gram_pmc_ab.sh r03g "GRF_BW=4096 GRF_SPLIT=0" "GRF_BW=4096 GRF_SPLIT=1" "GRF_BW=8192 GRF_SPLIT=0" "GRF_BW=8192 GRF_SPLIT=1" "GRF_BW=8192 GRF_SPLIT=1 GRF_GRAM_WAVES=4"
