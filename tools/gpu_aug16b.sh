#!/bin/bash
# C4 pipelined step with 16- vs 32-byte walk records (interleaved), then the walk kernel's FETCH_SIZE for each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/aug16b
mkdir -p $O
run() {
  env $1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$1 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['roofline_walk']['kernel_ms'],3), round(d['serial_ms_per_step'],2))")"
}
for i in 1 2 3; do run GRF_WALK_AUG16=0; run GRF_WALK_AUG16=1; done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  GRF_WALK_AUG16=$v timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-mfma-leg > $O/pmc$v.log 2>&1 || { echo pmc failed; tail $O/pmc$v.log; exit 1; }
  python3 - $O/pmc$v <<'PY'
import csv,glob,sys
f=glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True)[0]
tot={}
for r in csv.DictReader(open(f)):
    if 'phi_fused' in r['Kernel_Name']:
        tot.setdefault(r['Dispatch_Id'],0.0); tot[r['Dispatch_Id']]+=float(r['Counter_Value'])
print(sys.argv[1], 'phi_fused FETCH_SIZE KiB per launch', [round(v) for v in tot.values()])
PY
done
