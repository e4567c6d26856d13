set -o pipefail
mkdir -p gpurun_out/ab
i=0
for cfg in "GRF_BW=4096" "GRF_BW=3072" "GRF_BW=3584" "GRF_BW=2560" "GRF_BW=4096" "GRF_BW=3072"; do
  env $cfg timeout -k 10 300 python3 tools/gram_time.py 100000 5 sym > gpurun_out/ab/w$i.json 2> gpurun_out/ab/w$i.err || { echo "cfg $cfg failed"; tail -5 gpurun_out/ab/w$i.err; exit 1; }
  echo "$cfg: $(cat gpurun_out/ab/w$i.json)"
  i=$((i+1))
done
