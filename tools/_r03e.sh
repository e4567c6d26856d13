set -o pipefail
bash tools/gpu_ab.sh r03e "bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3" "X=0" "X=0 :: --front-split" "X=0 :: --front-split --mirror-wgs 0" "X=0 :: --front-split --mirror-wgs 1536"
