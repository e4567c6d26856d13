#!/bin/bash
# pipelined-window knobs with the self-counting transpose: mirror grid cap x next-front start
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02k
mkdir -p $O
run() {
  GRF_MIRROR_WGS=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --front-at $2 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "wgs=$1 front_at=$2 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2))")"
}
for w in 1024 1536 2048 0 768 1024; do run $w 1.0; done
for fa in 0.97 0.93 0.9; do run 1024 $fa; done
run 1536 0.95
