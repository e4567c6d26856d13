set -o pipefail
bash tools/gpu_tests.sh r04_ab14_tests "gram_dense or c3 or dense_steps or gpflow" 300 || exit 1
O=gpurun_out/r04_dense_ab14.txt
bash tools/gpu_dense_ab.sh $O "base base" 2708 4096 10000 16384 || exit 1
