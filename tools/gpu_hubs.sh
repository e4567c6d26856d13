#!/bin/bash
# hub-column split: parity tests, then Enron / Facebook / C4 bench lines over the number of hub columns
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/hubs
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_capi.py -x -v --timeout 200 --timeout-method thread \
    -k "hub or capi or export or symbol" > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for g in enron facebook; do
for h in ${HUB_LIST:-0 64 128 256 512}; do
  timeout -k 10 200 python bench.py --graph $g --steps 10 --warmup 2 --no-cpu-baseline --no-mfma-leg --hubs $h \
      > $O/${g}_h$h.json 2> $O/${g}_h$h.err || { echo "$g $h failed"; tail $O/${g}_h$h.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), 'K-assembly', round(d['roofline']['kernel_ms'],3), 'serial', round(d.get('serial_ms_per_step',0),3))" $O/${g}_h$h.json "$g hubs=$h"
done
done
