set -o pipefail
mkdir -p gpurun_out/r03n
for rep in 1 2; do
for cfg in "GRF_DENSE_DB=1" "GRF_DENSE_DB=0" "GRF_DENSE_DB=1 GRF_DENSE_BK=32" "GRF_DENSE_DB=0 GRF_DENSE_BK=32"; do
  env $cfg timeout -k 10 200 python3 tools/dense_sweep.py 2708 4096 10000 >> gpurun_out/r03n/sweep.txt 2>gpurun_out/r03n/sweep.err || { echo "cfg $cfg failed"; tail -5 gpurun_out/r03n/sweep.err; exit 1; }
done
done
cat gpurun_out/r03n/sweep.txt
bash tools/gpu_tests.sh r03n "dense" 600
