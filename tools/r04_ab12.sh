set -o pipefail
O=gpurun_out/r04_dense_ab12.txt
bash tools/gpu_dense_ab.sh $O "base GRF_DENSE_SK=1 GRF_DENSE_SK=1,GRF_DENSE_IL=1 base GRF_DENSE_SK=1" 2708 4096 10000 16384 || exit 1
bash tools/gpu_dense_ab.sh $O "base GRF_DENSE_SK=1" 1000 1500 6000 || exit 1
