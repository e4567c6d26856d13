#!/bin/bash
# kernel-trace stats of a short bench run -> gpurun_out/<tag>/trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-trace}; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $O/trace.log 2>&1 || { echo trace failed; tail $O/trace.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{float(r['AverageNs'])/1e6:8.3f} ms x{r['Calls']:>3}  {r['Name'][:90]}")
PY
