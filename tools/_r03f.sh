set -o pipefail
bash tools/gpu_tests.sh r03f "" 1000 && \
bash tools/gpu_profile.sh r03f && \
bash tools/gpu_ab.sh r03f_c5 "bench.py --workload c5 --no-cpu-baseline --steps 10 --warmup 2" "X=0 :: --hubs 0" "X=0 :: --hubs 16" "X=0 :: --hubs 64"
