set -o pipefail
mkdir -p gpurun_out/ab
i=0
for cfg in "GRF_GRAM_BAL=0" "GRF_GRAM_BAL=1" "GRF_GRAM_BAL=0" "GRF_GRAM_BAL=1"; do
  env $cfg timeout -k 10 300 python3 tools/gram_time.py 100000 5 sym,rows > gpurun_out/ab/b$i.json 2> gpurun_out/ab/b$i.err || { echo "cfg $cfg failed"; tail -5 gpurun_out/ab/b$i.err; exit 1; }
  echo "$cfg: $(cat gpurun_out/ab/b$i.json)"
  i=$((i+1))
done
