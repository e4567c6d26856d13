set -o pipefail
mkdir -p gpurun_out/wab
i=0
for cfg in "$@"; do
  for w in c4 c5; do
    env $cfg timeout -k 10 300 python3 tools/walkphi_ab.py $w > gpurun_out/wab/$i$w.json 2> gpurun_out/wab/$i$w.err || { echo "cfg $cfg $w failed"; tail -5 gpurun_out/wab/$i$w.err; exit 1; }
    echo "$cfg $w: $(cat gpurun_out/wab/$i$w.json)"
  done
  i=$((i+1))
done
