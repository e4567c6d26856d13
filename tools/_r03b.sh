set -o pipefail
bash tools/gpu_tests.sh r03b "sub_band_split or dense_steps or shift_bound or gpflow or gram_sparse_vs_oracle or staged_fill or block_symmetric or column_block or hub_column or degenerate or philox_vs_reference or bench_line_n2" 1000 && \
bash tools/gpu_ab.sh r03b "tools/gram_time.py 100000 5 upper,sym" "GRF_BW=4096 GRF_GRAM_SPLIT=0" "GRF_BW=4096 GRF_GRAM_SPLIT=1" "GRF_BW=8192 GRF_GRAM_SPLIT=0" "GRF_BW=8192 GRF_GRAM_SPLIT=1" && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err && tail -c 700 gpurun_out/r03b/bench.json
