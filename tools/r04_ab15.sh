#!/bin/bash
# A/B: the hub panel's ring (GRF_DENSE_HUB_NST 4 = two 64 KB workgroups per CU, 3 = three 48 KB) on the
# Enron and Facebook benches (alternating arms), then a kernel trace of Enron under arm 3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_ab15
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in enron facebook; do
  for rep in 1 2; do
    for nst in 4 3; do
      GRF_DENSE_HUB_NST=$nst timeout -k 10 240 python3 $R/bench.py --graph $g --steps 10 --warmup 2 --no-cpu-baseline \
          --no-mfma-leg > $O/${g}_nst${nst}_$rep.json 2> $O/${g}_nst${nst}_$rep.err || { echo "$g nst$nst failed"; tail $O/${g}_nst${nst}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" \
          $O/${g}_nst${nst}_$rep.json "$g nst=$nst rep=$rep"
    done
  done
done
export GRF_DENSE_HUB_NST=3
for h in 128 160; do  # (a faster panel may pay for more hub columns)
  timeout -k 10 240 python3 $R/bench.py --graph enron --hubs $h --steps 10 --warmup 2 --no-cpu-baseline --no-mfma-leg \
      > $O/enron_nst3_h$h.json 2> $O/enron_nst3_h$h.err || { echo "hubs $h failed"; tail $O/enron_nst3_h$h.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" \
      $O/enron_nst3_h$h.json "enron nst=3 hubs=$h"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --graph enron --steps 10 --warmup 2 --no-cpu-baseline --no-mfma-leg > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
echo trace ok
