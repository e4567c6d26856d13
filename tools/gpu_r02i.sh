#!/bin/bash
# dense MFMA Gram (C3) tile / k-tile A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02i
mkdir -p $O
for cfg in "0 0" "128 32" "128 64" "64 32" "128 64" "0 0"; do
  set -- $cfg
  GRF_DENSE_TILE=$1 GRF_DENSE_BK=$2 timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --steps 50 > $O/c3.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "tile=$1 bk=$2 $(python -c "import json;d=json.loads(open('$O/c3.json').read().splitlines()[-1]);r=d['roofline'];print(round(d['ms_per_step'],3), round(r['kernel_ms'],4), round(r['achieved'],1), round(r['frac'],3))")"
done
