#!/bin/bash
# C5 column-block Gram decomposition (timing-only builds, K wrong): exp1 = no accumulation (zero + write-out),
# exp2 = no write-out (zero + accumulation); rocprofv3 kernel stats of the Gram under each
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c5decomp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in base exp1 exp2; do
  L=$R/efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so
  [ $v != base ] && L=$R/tools/libgrf_$v.so
  GRF_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-mfma-leg --workload c5 --steps 5 --warmup 2 --no-overlap > $O/$v.log 2>&1 || { echo $v failed; tail -5 $O/$v.log; exit 1; }
  python3 - $O/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gram' in r['Name'] or 'phi_fused' in r['Name']:
        print(sys.argv[1].split('/')[-1], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
