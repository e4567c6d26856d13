#!/bin/bash
# VALU / SALU / LDS instructions per wave of phi_fused_kernel: whole kernel vs walks only vs walks + sort
# (timing-only builds tools/libgrf_pexp{1,2}.so), C4 and C5, one --pmc pass each
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/phivalu
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in kernel c5; do
for v in ${PHI_VARIANTS:-base pexp1 pexp2}; do
  L=$R/efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so
  [ $v != base ] && L=$R/tools/libgrf_$v.so
  GRF_AMD_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/$w$v -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-mfma-leg --workload $w --steps 1 --warmup 0 --no-overlap > $O/$w$v.log 2>&1 || { echo $w $v failed; tail -5 $O/$w$v.log; exit 1; }
  python3 - $O/$w$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if 'phi_fused' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
c = {k: v / n[k] for k, v in acc.items()}
w = c['SQ_WAVES']
print(sys.argv[1].split('/')[-1], 'waves', int(w), {k: round(v / w) for k, v in c.items() if k != 'SQ_WAVES'})
PY
done
done
