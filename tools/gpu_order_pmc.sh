#!/bin/bash
# L2 hit rate and fetch of the Gram under GRF_GRAM_ORDER 0 / 2 (one --pmc pass each, no trace domains)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/order_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for o in 0 2; do
  GRF_GRAM_ORDER=$o timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/o$o -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-mfma-leg --steps 3 --warmup 1 > $O/o$o.log 2>&1 || { echo pass $o failed; tail -20 $O/o$o.log; exit 1; }
  python3 - $O/o$o <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if 'gram_sparse' not in k: continue
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, d in acc.items():
    c = {m: v / n[(k, m)] for m, v in d.items()}
    print(sys.argv[1].split('/')[-1], k[:50], {m: round(v) for m, v in c.items()},
          'hit', round(c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']), 3))
PY
done
# transpose placing pass with XCD-contiguous regions: parity, then prev / new library A/B (order 0)
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "transpose or bench_path or column_block or degenerate" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {
  env GRF_AMD_LIB=$1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-mfma-leg --steps 20 --warmup 3 > $O/b.json 2>> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "$2 $(python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(round(d['ms_per_step'],2), round(d['roofline']['kernel_ms'],2), round(d['serial_ms_per_step'],2))")"
}
for i in 1 2 3; do run tools/libgrf_prev.so prev; run efficient-gaussian-process-on-graphs_amd/grf_amd/libgrf_amd.so new; done
