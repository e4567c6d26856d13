# A/B of gram knobs: tools/gpu_gram_ab.sh "<ENV=val ...>" "<ENV=val ...>" ...
set -o pipefail
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python3 tools/gram_time.py 100000 5 > gpurun_out/ab/$i.json 2> gpurun_out/ab/$i.err || { echo "cfg $cfg failed"; tail -5 gpurun_out/ab/$i.err; exit 1; }
  echo "$cfg: $(cat gpurun_out/ab/$i.json)"
  i=$((i+1))
done
