#!/bin/bash
# pipelined C4 step vs the mirror's grid beside the next front (GRF_MIRROR_WGS; 1024 = default), after the walk_phi changes
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/mwgs2
mkdir -p $O
cd $R
for rep in 1 2; do
for w in 1024 768 1536 2048; do
  GRF_MIRROR_WGS=$w timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-mfma-leg > $O/w${w}_$rep.json 2> $O/w${w}_$rep.err || { echo "wgs $w failed"; tail $O/w${w}_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), 'K-assembly', round(d['roofline']['kernel_ms'],3))" $O/w${w}_$rep.json "mirror_wgs=$w rep=$rep"
done
done
