set -o pipefail
mkdir -p gpurun_out/r03a
for bw in 4096 8192; do
  GRF_BW=$bw timeout -k 10 300 python3 tools/gram_time.py 100000 5 sym,mirror > gpurun_out/r03a/bw$bw.json 2> gpurun_out/r03a/bw$bw.err || { echo "bw $bw failed"; tail -5 gpurun_out/r03a/bw$bw.err; exit 1; }
  echo "bw $bw: $(cat gpurun_out/r03a/bw$bw.json)"
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err && cat gpurun_out/r03a/bench.json
