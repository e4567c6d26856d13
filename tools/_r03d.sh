set -o pipefail
bash tools/gpu_tests.sh r03d "column_block_hub or c5_column_block_with_hub or sparse_api_philox or gpflow or dense_steps" 900 && \
bash tools/gpu_ab.sh r03d "bench.py --workload c5 --no-cpu-baseline --steps 10 --warmup 2" "X=0 :: --hubs 0" "X=0 :: --hubs 16" "X=0 :: --hubs 32" "X=0 :: --hubs 64"
