set -o pipefail
mkdir -p gpurun_out/ab
i=0
for cfg in "GRF_BW=8192" "GRF_BW=8192 GRF_GRAM_UNROLL=4" "GRF_BW=8192 GRF_GRAM_UNROLL=16" "GRF_BW=8192" "GRF_BW=8192 GRF_GRAM_UNROLL=4"; do
  env $cfg timeout -k 10 300 python3 tools/gram_time.py 100000 5 rows > gpurun_out/ab/u$i.json 2> gpurun_out/ab/u$i.err || { echo "cfg $cfg failed"; tail -5 gpurun_out/ab/u$i.err; exit 1; }
  echo "$cfg: $(cat gpurun_out/ab/u$i.json)"
  i=$((i+1))
done
