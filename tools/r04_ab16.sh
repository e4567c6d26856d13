#!/bin/bash
# Hub-column count sweep with the three-workgroup hub panel: Facebook (auto = 0) and Enron (auto = 96).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_ab16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for arm in facebook:0 facebook:32 facebook:64 enron:64 enron:96 facebook:32 enron:64 enron:96; do
  g=${arm%%:*}; h=${arm##*:}
  timeout -k 10 240 python3 $R/bench.py --graph $g --hubs $h --steps 10 --warmup 2 --no-cpu-baseline --no-mfma-leg \
      > $O/${g}_h$h.json 2> $O/${g}_h$h.err || { echo "$arm failed"; tail $O/${g}_h$h.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['config'].get('hub_columns'))" \
      $O/${g}_h$h.json "$g hubs=$h"
done
