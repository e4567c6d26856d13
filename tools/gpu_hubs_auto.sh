#!/bin/bash
# bench --hubs auto on Enron / Facebook / C4 against --hubs 0
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/hubsauto
mkdir -p $O
cd $R
for g in enron facebook er; do
for h in 0 auto; do
  timeout -k 10 200 python bench.py --graph $g --steps 10 --warmup 2 --no-cpu-baseline --no-mfma-leg --hubs $h \
      > $O/${g}_$h.json 2> $O/${g}_$h.err || { echo "$g $h failed"; tail $O/${g}_$h.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), 'hub_columns', d['config'].get('hub_columns'))" $O/${g}_$h.json "$g hubs=$h"
done
done
