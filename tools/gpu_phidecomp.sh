#!/bin/bash
# walk_phi decomposition (timing-only builds: rows left empty): pexp1 = walks only, pexp2 = walks + sort;
# rocprofv3 kernel stats of phi_fused_kernel, C4 and C5 serial steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/phidecomp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in kernel c5; do
for v in base pexp1 pexp2; do
  L=$R/efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so
  [ $v != base ] && L=$R/tools/libgrf_$v.so
  GRF_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$w$v -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-mfma-leg --workload $w --steps 4 --warmup 1 --no-overlap > $O/$w$v.log 2>&1 || { echo $w $v failed; tail -5 $O/$w$v.log; exit 1; }
  python3 - $O/$w$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'phi_fused' in r['Name']:
        print(sys.argv[1].split('/')[-1], r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e6, 3))
PY
done
done
